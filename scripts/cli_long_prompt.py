"""`dllama inference` on a ~4096-token prompt at default flags (--prefill-chunk defaults to 1024
on GPUs): prints the reference's Evaluation / Prediction summary lines. Synthetic Llama-3.1-8B
weights, synthetic tokenizer (byte fallback: ~1 token per character)."""
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_llama_multiusers_amd.models.synthetic import make_tokenizer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
with tempfile.TemporaryDirectory() as d:
    tok = os.path.join(d, "llama3_synth.t")
    make_tokenizer(tok, 128256)
    prompt = ("The quick brown fox jumps over the lazy dog " * (n // 44 + 1))[:n]
    cmd = [os.path.join(REPO, "build", "dllama"), "inference", "--synthetic", "llama3_1_8b", "--tokenizer", tok,
           "--prompt", prompt, "--steps", str(n + 32), "--temperature", "0", "--gpu-index", "0",
           "--max-seq-len", str(n + 64), "--buffer-float-type", "q80", "--log-level", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if "tokens/s" in l or "Evaluation" in l or "Prediction" in l
             or "nTokens" in l]
    print("\n".join(lines[-8:]))
    print("rc", r.returncode, r.stderr[-500:] if r.returncode else "")
