#!/usr/bin/env python3
"""Register-safety check of the ring GEMV kernels: the weight ring and the exchange epochs
are loaded with inline asm, so the compiler does not know those VGPRs are pending; a spill or a copy
of them before their s_waitcnt would read stale data. Every gemvQ40Kernel / attnBlockKernel instance
must therefore compile with no scratch (no spills) - checked from hipcc's resource-usage remarks.

    python scripts/check_isa.py            # make check-isa
"""
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

SRCS = ["csrc/hip/gemv_l16.hip", "csrc/hip/gemv_l32.hip", "csrc/hip/gemv_l64.hip", "csrc/hip/attn_block_16_32_128.hip",
        "csrc/hip/attn_block_64_64_128.hip", "csrc/hip/attn_block_64_64_64.hip", "csrc/hip/ffn_block.hip"]
FLAGS = ["-std=c++17", "-O3", "--offload-arch=gfx950", "-munsafe-fp-atomics", "--offload-device-only", "-c",
         "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]


def check(src):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, src], capture_output=True, text=True)
    if r.returncode != 0:
        return src, [f"compile failed: {r.stderr[-500:]}"], 0
    bad, fn, n = [], None, 0
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            fn = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and fn and ("gemvQ40Kernel" in fn or "attnBlockKernel" in fn or "gemvAttnKernel" in fn or "ffnBlockKernel" in fn):
            n += 1
            if int(m.group(1)) != 0:
                bad.append(f"{fn}: scratch {m.group(1)} B/lane")
    return src, bad, n


def main():
    with ThreadPoolExecutor(4) as ex:
        res = list(ex.map(check, SRCS))
    ok = True
    for src, bad, n in res:
        print(f"{src}: {n} ring-kernel instances, {len(bad)} with scratch")
        for b in bad:
            print("  " + b)
        ok = ok and not bad and n > 0
    return 0 if ok else 1


if __name__ == "__main__" and "--hazards" not in sys.argv:
    sys.exit(main())


# ---- pending-register hazard scan: an instruction that READS a VGPR whose inline-asm
# load is still outstanding (no s_waitcnt vmcnt has retired it yet) sees the old value: gfx9 has no
# VMEM interlock. Linear scan of each kernel's assembly (fall-through order), counting every VMEM
# instruction against vmcnt as the hardware does (gfx9: loads and stores).
VMEM = re.compile(r"^\s*(global|buffer|scratch|flat)_(load|store|atomic)\S*")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def scan_asm(path, want):
    hazards = []
    lines = open(path).read().splitlines()
    fn, q, in_asm = None, [], False
    for ln in lines:
        if re.match(r"^_ZN\S+:", ln):
            fn, q, in_asm = ln.split(":")[0], [], False
            continue
        if fn is None or not any(w in fn for w in want):
            continue
        s = ln.split(";")[0].strip()
        if ";;#ASMSTART" in ln:
            in_asm = True
            continue
        if ";;#ASMEND" in ln:
            in_asm = False
            continue
        if not s or s.endswith(":") or s.startswith("."):
            continue
        if s.startswith("s_endpgm"):
            fn = None
            continue
        m = re.match(r"s_waitcnt\s+(.*)", s)
        if m:
            v = re.search(r"vmcnt\((\d+)\)", m.group(1))
            if v:
                while len(q) > int(v.group(1)):
                    q.pop(0)
            continue
        ops = s.split(None, 1)
        op, args = ops[0], ops[1] if len(ops) > 1 else ""
        parts = [p.strip() for p in args.split(",")]
        if VMEM.match(s):
            is_load = "_load" in op or ("atomic" in op and " glc" in s)
            dst = regs(parts[0]) if is_load else set()
            srcs = regs(",".join(parts[1:] if is_load else parts))
        elif op.startswith("v_") or op.startswith("ds_") or op.startswith("s_"):
            dst = set()
            srcs = regs(",".join(parts[1:])) if (op.startswith("v_") or op.startswith("ds_read")) else regs(",".join(parts))
        else:
            continue
        pend = set()
        for d, asm in q:
            if asm:
                pend |= d
        bad = srcs & pend
        if bad:
            hazards.append(f"{fn[:60]}: '{s}' reads pending v{sorted(bad)}")
        if VMEM.match(s):
            q.append((dst, in_asm))
    return hazards


def hazard_check():
    import glob
    import os
    import tempfile
    ok = True
    with tempfile.TemporaryDirectory() as d:
        for src in ["csrc/hip/gemv_l16.hip", "csrc/hip/gemv_l32.hip", "csrc/hip/gemv_l64.hip", "csrc/hip/attn_block_16_32_128.hip",
                    "csrc/hip/ffn_block.hip"]:
            r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS[:5], "--save-temps", "-c", "-o", os.path.join(d, "x.o"),
                                os.path.abspath(src)], capture_output=True, text=True, cwd=d)
            s_files = glob.glob(os.path.join(d, "*gfx950.s"))
            if r.returncode != 0 or not s_files:
                print(f"{src}: no assembly ({r.stderr[-300:]})")
                return False
            hz = scan_asm(s_files[0], ["gemvQ40Kernel", "attnBlockKernel", "gemvAttnKernel", "ffnBlockKernel"])
            print(f"{src}: {len(hz)} reads of pending inline-asm load registers")
            for h in hz[:20]:
                print("  " + h)
            ok = ok and not hz
            for f in glob.glob(os.path.join(d, "*")):
                os.remove(f)
    return ok


if __name__ == "__main__" and "--hazards" in sys.argv:
    sys.exit(0 if hazard_check() else 1)
