#!/usr/bin/env python3
"""The lane-pair PLL step's ISA with its dependent chain marked.

Disassembles k_pll_multi<VEC, SPLIT, WG = 1> from a device-only build of sdr_pll.hip, finds the
unrolled fast 16-step chunk of the trigArg-table path (the basic block with 16 v_bitop3_b32, one
per step), builds the VGPR def-use graph of the chunk (64-bit operands as register pairs, DPP and
op_sel sources included) and reports:
  * VALU / SALU / LDS / s_nop per step, and f64 operations per step by kind;
  * the longest dependence chain through the chunk (the recurrence: 16 steps deep), per step;
  * one step's listing with each instruction marked [f64] and [chain] (on a longest path).
  python tools/pll_isa.py [--out profiles/r04/pll_step_isa.txt]
"""
from __future__ import annotations

import argparse
import pathlib
import re
import subprocess
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
         "-mllvm", "-pragma-unroll-threshold=1000000", "-fno-slp-vectorize", "-I", str(ROOT / "include"),
         "-mllvm", "-amdgpu-sched-strategy=max-ilp", "--cuda-device-only", "--no-gpu-bundle-output", "-c"]
F64 = re.compile(r"^v_(fma|fmac|add|mul|cvt_f32_f64|cvt_f64_f32|cvt_f64_i32|fract|rndne)_f64|^v_cvt_f(32|64)_f(64|32)|^v_cvt_f64_i32")


def regs(tok: str) -> list[str]:
    """VGPR names of one operand (v5, v[4:5], -v[0:1], |v3|)."""
    tok = tok.strip().lstrip("-|").rstrip("|")
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return [f"v{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)]
    m = re.match(r"v(\d+)$", tok)
    return [f"v{m.group(1)}"] if m else []


def parse(line: str):
    s = line.split("//")[0].strip()
    if not s or s.endswith(":"):
        return None
    parts = s.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])] if len(parts) > 1 else []
    mods = ops[-1].split()[1:] if ops else []
    if ops:
        ops[-1] = ops[-1].split()[0] if ops[-1].split() else ops[-1]
    return op, ops, mods, s


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--extra", default="", help="extra compiler flags (scheduler A/B)")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        obj = pathlib.Path(d) / "pll.o"
        subprocess.run([HIPCC, *FLAGS, *args.extra.split(), "-o", str(obj), str(ROOT / "real-time-sdr_amd/csrc/sdr_pll.hip")],
                       check=True)
        dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(obj)], capture_output=True, text=True,
                             check=True).stdout
    lines = dis.split("\n")
    start = next(i for i, l in enumerate(lines) if re.search(r"<.*k_pll_multiILb1ELb1ELi1ELb0E.*>:", l))
    end = next(i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <.*>:$", lines[i].strip()))
    # basic blocks of the kernel; the TAB fast chunk: 16 bitop3 and 8 ds_read_b128 (the table)
    blocks, cur = [], []
    for l in lines[start + 1:end]:
        p = parse(l)
        if p is None:
            continue
        cur.append(p)
        if re.match(r"s_(cbranch|branch)", p[0]):
            blocks.append(cur)
            cur = []
    # (16 more bitop3 with the base-angle table of SDR_PLL_BASETAB)
    chunk = next(b for b in blocks if sum(x[0] == "v_bitop3_b32" for x in b) in (16, 32)
                 and sum(x[0] == "ds_read_b128" for x in b) >= 8)
    steps = 16
    cnt = {"VALU": 0, "SALU": 0, "LDS": 0, "s_nop": 0, "VMEM": 0}
    f64 = {}
    for op, _, _, _ in chunk:
        if op == "s_nop":
            cnt["s_nop"] += 1
        elif op.startswith("v_"):
            cnt["VALU"] += 1
            if F64.match(op):
                f64[op] = f64.get(op, 0) + 1
        elif op.startswith("s_"):
            cnt["SALU"] += 1
        elif op.startswith("ds_"):
            cnt["LDS"] += 1
        elif op.startswith(("global_", "buffer_")):
            cnt["VMEM"] += 1
    # def-use graph (VALU only; the first operand is the destination of every VALU form used here)
    last_def: dict[str, int] = {}
    depth = [0] * len(chunk)
    pred = [-1] * len(chunk)
    for i, (op, ops, mods, _) in enumerate(chunk):
        if not op.startswith("v_") or not ops:
            continue
        srcs = [r for o in ops[1:] for r in regs(o)]
        if op.startswith(("v_fmac_", "v_mac_")):
            srcs += regs(ops[0])                      # the accumulator is read too
        best, arg = 0, -1
        for r in srcs:
            j = last_def.get(r)
            if j is not None and depth[j] + 1 > best:
                best, arg = depth[j] + 1, j
        depth[i] = max(best, 1)
        pred[i] = arg
        for r in regs(ops[0]):
            last_def[r] = i
    tail = max(range(len(chunk)), key=lambda i: depth[i])
    chain = set()
    i = tail
    while i >= 0:
        chain.add(i)
        i = pred[i]
    # one step in the middle of the chunk: between the 8th and 9th v_bitop3
    bops = [i for i, x in enumerate(chunk) if x[0] == "v_bitop3_b32"]
    lo, hi = bops[7] + 1, bops[8] + 1
    out = []
    out.append("k_pll_multi<VEC, SPLIT, WG = 1>, trigArg-table fast chunk (16 unrolled lane-pair steps), "
               "gfx950, from tools/pll_isa.py")
    out.append("per step: " + ", ".join(f"{k} {v / steps:.2f}" for k, v in cnt.items()))
    out.append("f64 ops per step: " + ", ".join(f"{k} {v / steps:.2f}" for k, v in sorted(f64.items())) +
               f" (total {sum(f64.values()) / steps:.2f})")
    out.append(f"longest VGPR dependence chain through the chunk: {depth[tail]} VALU levels = "
               f"{depth[tail] / steps:.2f} per step (the step's recurrence)")
    out.append("")
    out.append("one step (marks: [f64] double-precision or f32<->f64 conversion, [chain] on the longest path):")
    for i in range(lo, hi):
        op, _, _, text = chunk[i]
        mark = ("[f64]" if F64.match(op) else "     ") + (" [chain]" if i in chain else "        ")
        out.append(f"  {mark}  {text}")
    txt = "\n".join(out) + "\n"
    if args.out:
        pathlib.Path(args.out).write_text(txt)
    print(txt)


if __name__ == "__main__":
    main()
