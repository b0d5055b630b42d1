#!/usr/bin/env python3
"""Download a published distributed-llama model and write a run script (reference: launch.py).

    python launch.py <model> [--gpus N] [--api] [--cpu] [--run] [--yes] [--no-download]

Unlike the reference (which writes one CPU `dllama chat` line), the run script starts one
process per GPU: N-1 `dllama worker` processes pinned with --gpu-index 1..N-1 and the root on
GPU 0, tensor-parallel over RCCL; workers are stopped by PID when the root exits.
Downloads resume from the last complete part and retry each part up to 8 times.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from dataclasses import dataclass, field
from typing import List
from urllib.request import urlopen

HF = "https://huggingface.co/b4rtaz"


def _parts(n: int) -> List[str]:
    return [chr(97 + i // 26) + chr(97 + i % 26) for i in range(n)]


@dataclass
class ModelEntry:
    urls: List[str]
    tokenizer_url: str
    weights: str = "q40"
    buffer: str = "q80"
    mode: str = "chat"
    extra: List[str] = field(default_factory=lambda: ["--max-seq-len", "4096"])


def _single(repo: str, model: str, tok: str) -> ModelEntry:
    base = f"{HF}/{repo}/resolve/main"
    return ModelEntry([f"{base}/{model}?download=true"], f"{base}/{tok}?download=true")


def _split(repo: str, prefix: str, n: int, tok: str) -> ModelEntry:
    base = f"{HF}/{repo}/resolve/main"
    return ModelEntry([f"{base}/{prefix}{s}?download=true" for s in _parts(n)], f"{base}/{tok}?download=true")


MODELS = {
    "llama3_1_8b_instruct_q40": _single("Llama-3_1-8B-Q40-Instruct-Distributed-Llama",
                                        "dllama_model_llama3.1_instruct_q40.m", "dllama_tokenizer_llama_3_1.t"),
    "llama3_1_405b_instruct_q40": _split("Llama-3_1-405B-Q40-Instruct-Distributed-Llama",
                                         "dllama_model_llama31_405b_q40_", 56, "dllama_tokenizer_llama_3_1.t"),
    "llama3_2_1b_instruct_q40": _single("Llama-3_2-1B-Q40-Instruct-Distributed-Llama",
                                        "dllama_model_llama3.2-1b-instruct_q40.m", "dllama_tokenizer_llama3_2.t"),
    "llama3_2_3b_instruct_q40": _single("Llama-3_2-3B-Q40-Instruct-Distributed-Llama",
                                        "dllama_model_llama3.2-3b-instruct_q40.m", "dllama_tokenizer_llama3_2.t"),
    "llama3_3_70b_instruct_q40": _split("Llama-3_3-70B-Q40-Instruct-Distributed-Llama",
                                        "dllama_model_llama-3.3-70b_q40", 11, "dllama_tokenizer_llama-3.3-70b.t"),
    "deepseek_r1_distill_llama_8b_q40": _single("DeepSeek-R1-Distill-Llama-8B-Distributed-Llama",
                                                "dllama_model_deepseek-r1-distill-llama-8b_q40.m",
                                                "dllama_tokenizer_deepseek-r1-distill-llama-8b.t"),
}


def confirm(msg: str, yes: bool) -> bool:
    if yes:
        return True
    return input(f'{msg} ("Y" if yes): ').strip().upper() in ("Y", "YES")


def download(urls: List[str], path: str, yes: bool) -> None:
    if os.path.isfile(path) and not confirm(f"{os.path.basename(path)} already exists, download again?", yes):
        return
    with open(path, "wb") as f:
        for url in urls:
            start = f.tell()
            for attempt in range(8):
                print(f"{url} (attempt: {attempt})")
                try:
                    with urlopen(url) as r:
                        last = -1
                        while chunk := r.read(1 << 20):
                            f.write(chunk)
                            mb = f.tell() >> 20
                            if mb // 64 != last:
                                sys.stdout.write(f"\rDownloaded {mb} MB")
                                last = mb // 64
                    sys.stdout.write("\n")
                    break
                except Exception as e:  # network errors: rewind this part and retry
                    print(f"\nError downloading {url}: {e}")
                    f.seek(start)
                    f.truncate()
                    time.sleep(attempt)
            else:
                raise RuntimeError(f"Failed to download {url}")


def run_command(name: str, e: ModelEntry, model: str, tok: str, gpus: int, api: bool, cpu: bool) -> str:
    exe = "build/dllama-api" if api else "build/dllama"
    mode = "" if api else ("chat" if e.mode == "chat" else 'inference --steps 64 --prompt "Hello world"')
    common = f"--model {model} --tokenizer {tok} --buffer-float-type {e.buffer} {' '.join(e.extra)}"
    lines = ["#!/bin/bash", "set -e", 'cd "$(dirname "$0")"', "export HSA_ENABLE_IPC_MODE_LEGACY=0"]
    if cpu:
        lines.append(f"{exe} {mode} {common} --nthreads {os.cpu_count()} \"$@\"")
        return "\n".join(lines) + "\n"
    workers = []
    if gpus > 1:
        lines.append("PIDS=()")
        lines.append('trap \'for p in "${PIDS[@]}"; do kill "$p" 2>/dev/null || true; done\' EXIT')
        for g in range(1, gpus):
            port = 9998 - g
            workers.append(f"127.0.0.1:{port}")
            lines.append(f"build/dllama worker --port {port} --gpu-index {g} > worker_{g}.log 2>&1 &")
            lines.append("PIDS+=($!)")
        lines.append("sleep 2")
    w = f" --workers {' '.join(workers)}" if workers else ""
    lines.append(f"{exe} {mode} {common} --gpu-index 0{w} \"$@\"")
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    cwd = os.getcwd()
    try:
        return _main(argv)
    finally:
        os.chdir(cwd)


def _main(argv) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("model", nargs="?")
    ap.add_argument("--gpus", type=int, default=1, help="tensor-parallel degree (one process per GPU)")
    ap.add_argument("--api", action="store_true", help="write a dllama-api run script")
    ap.add_argument("--cpu", action="store_true", help="run on the CPU backend")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--yes", action="store_true", help="answer yes to all prompts")
    ap.add_argument("--no-download", action="store_true", help="only write the run script")
    ap.add_argument("--dir", default=os.path.dirname(os.path.abspath(__file__)))
    a = ap.parse_args(argv)
    if not a.model:
        ap.print_help()
        print("\nAvailable models:\n" + "\n".join(f"  {m}" for m in MODELS))
        return 1
    name = a.model.replace("-", "_")
    if name not in MODELS:
        print(f"Model is not supported: {name}")
        return 1
    e = MODELS[name]
    d = os.path.join("models", name)
    model, tok = os.path.join(d, f"dllama_model_{name}.m"), os.path.join(d, f"dllama_tokenizer_{name}.t")
    os.chdir(a.dir)
    if not a.no_download:
        os.makedirs(d, exist_ok=True)
        print(f"Downloading {name} to {d}...")
        download(e.urls, model, a.yes)
        download([e.tokenizer_url], tok, a.yes)
        print("All files are downloaded")
    script = run_command(name, e, model, tok, a.gpus, a.api, a.cpu)
    path = f"run_{name}{'_api' if a.api else ''}{f'_tp{a.gpus}' if a.gpus > 1 else ''}.sh"
    with open(path, "w") as f:
        f.write(script)
    os.chmod(path, 0o755)
    print(f"--- {path} ---\n{script}---")
    if a.run or (not a.no_download and confirm("Do you want to run it now?", a.yes)):
        if not os.path.isfile("build/dllama"):
            import subprocess
            subprocess.check_call(["make", "-j8", "all"])
        import subprocess
        return subprocess.call(["bash", path])
    return 0


if __name__ == "__main__":
    sys.exit(main())
