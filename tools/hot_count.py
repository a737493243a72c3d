"""Static instruction count of the run kernel's common path (CPU only).

Compiles csrc/rwrt.hip for gfx950 with -DRWRT_ANALYZE_HOT, which turns every
rarely taken branch (RARE(...) in rwrt.hip, NM_RARE in np_math.h) and the
latency mode into dead code: the ray loop of rk45_run_kernel is then its
common path, so its static instruction count is what a wave issues per attempt
(plus the once-per-interval post-processing and the cell-cache refill, both
branches, reported separately).  Used to A/B instruction-count changes without
a GPU; the product build is unaffected.

  python tools/hot_count.py [--defs "-DX=1 ..."] [--kernel static|c5_64|c5_32] [--asm out.s]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rossby-wave-ray-tracing_amd", "csrc")
KERNELS = {
    "static": "_ZN4rwrt15rk45_run_kernelINS_8StaticBGELb0EEEvNS_7RunArgsIT_EE",
    "c5_64": "_ZN4rwrt15rk45_run_kernelINS_9VaryingBGIdEELb0EEEvNS_7RunArgsIT_EE",
    "c5_32": "_ZN4rwrt15rk45_run_kernelINS_9VaryingBGIfEELb0EEEvNS_7RunArgsIT_EE",
}


def compile_asm(defs, out):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fno-fast-math", "-fconstexpr-steps=20000000", "-I" + os.path.join(ROOT, "include"),
           "--cuda-device-only", "-S", "-DRWRT_ANALYZE_HOT", *defs, "-o", out,
           os.path.join(CSRC, "rwrt.hip")]
    subprocess.run(cmd, check=True)


def kernel_lines(asm, name):
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def blocks(lines):
    """(label, instructions) of each basic block"""
    bl, cur = [], ["entry", []]
    for l in lines:
        s = l.strip()
        if (s.startswith(".LBB") and s.split(";")[0].strip().endswith(":")) or s.startswith("; %bb."):
            bl.append(cur)
            cur = [s.split(":")[0].replace("; ", ""), []]
            continue
        if not s or s.startswith((".", ";")):
            continue
        cur[1].append(s)
    bl.append(cur)
    return bl


def klass(op):
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        return "spill_lane"
    if op.startswith("v_accvgpr"):
        return "agpr_move"
    if op.startswith(("v_mov_b64", "v_mov_b32")) and "dpp" not in op:
        return "vmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith(("s_waitcnt", "s_barrier", "s_sched", "s_setprio", "s_endpgm", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def count(lines):
    c = collections.Counter()
    ops = collections.Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c[klass(op)] += 1
        ops[op] += 1
    return c, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--defs", default="")
    ap.add_argument("--kernel", default="static", choices=sorted(KERNELS))
    ap.add_argument("--asm", default=None, help="keep the assembly here")
    ap.add_argument("--top", type=int, default=0, help="print the N most frequent opcodes")
    args = ap.parse_args()
    out = args.asm or os.path.join(tempfile.gettempdir(), "rwrt_hot.s")
    compile_asm(args.defs.split(), out)
    lines = kernel_lines(out, KERNELS[args.kernel])
    c, ops = count(lines)
    # the attempt's straight-line blocks: every block of > 300 instructions
    # (the six stage evaluations, the last one with the step control)
    big = [(n, ins) for n, ins in blocks(lines) if len(ins) > 300]
    attempt = collections.Counter()
    for _, ins in big:
        for i in ins:
            attempt[klass(i.split()[0])] += 1
    total = sum(c.values())
    issue = total - c["wait"]
    meta = "\n".join(lines[-0:])
    print(f"kernel {args.kernel} defs '{args.defs}'")
    print(f"  instructions {total}  (issue-slot {issue})  " +
          "  ".join(f"{k} {c[k]}" for k in ("valu", "vmov", "spill_lane", "agpr_move", "salu", "s_nop",
                                              "lds", "vmem", "wait", "other")))
    at = sum(attempt.values())
    print(f"  attempt blocks {len(big)}: {at} (issue-slot {at - attempt['wait']})  " +
          "  ".join(f"{k} {attempt[k]}" for k in ("valu", "vmov", "spill_lane", "agpr_move", "salu", "s_nop",
                                                    "lds", "vmem", "wait")) +
          "  sizes " + " ".join(str(len(ins)) for _, ins in big))
    txt = open(out).read()
    m = re.search(re.escape(KERNELS[args.kernel]) + r"[\s\S]*?\.vgpr_count:\s+(\d+)", txt)
    for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count"):
        mm = re.search(r"\.name:\s+" + re.escape(KERNELS[args.kernel]) + r"[\s\S]*?\." + key + r":\s+(\d+)", txt)
        mm = mm or re.search(r"\." + key + r":\s+(\d+)[\s\S]*?\.name:\s+" + re.escape(KERNELS[args.kernel]) + r"\n", txt)
        if mm:
            print(f"  {key} {mm.group(1)}")
    if args.top:
        for op, n in ops.most_common(args.top):
            print(f"    {n:6d} {op}")


if __name__ == "__main__":
    main()
