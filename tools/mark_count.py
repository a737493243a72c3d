"""Instructions between consecutive MARK points of an analysis build (CPU only).

    python tools/mark_count.py [--defs "-DRWRT_ANALYZE_QUAD"] [--asm out.s]

Compiles csrc/rwrt.hip with -DRWRT_ANALYZE_HOT -DRWRT_ANALYZE_MARK (+ --defs)
and prints, for the run kernel, the instruction classes between each pair of
consecutive "@MARK" comments in layout order -- where an attempt's issue
slots go, section by section (the rare branches are dead code there)."""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hot_count as hc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--defs", default="")
    ap.add_argument("--kernel", default="static", choices=sorted(hc.KERNELS))
    ap.add_argument("--asm", default="/tmp/rwrt_mark.s")
    a = ap.parse_args()
    hc.compile_asm(["-DRWRT_ANALYZE_MARK"] + a.defs.split(), a.asm)
    lines = hc.kernel_lines(a.asm, hc.KERNELS[a.kernel])
    cur, sec = "entry", collections.OrderedDict()
    order = []
    for l in lines:
        s = l.strip()
        if "@MARK" in s:
            cur = s.split("@MARK")[1].strip()
            order.append(cur)
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        sec.setdefault(cur, collections.Counter())[hc.klass(s.split()[0])] += 1
    tot = collections.Counter()
    print(f"{'section (after mark)':28s} {'all':>6s} " + " ".join(f"{k:>6s}" for k in
          ("valu", "vmov", "salu", "lds", "s_nop", "spill_lane", "agpr_move")))
    seen = set()
    for k in order:
        if k in seen:
            continue
        seen.add(k)
        c = sec.get(k, collections.Counter())
        n = sum(c.values()) - c["wait"]
        tot += c
        print(f"{k:28s} {n:6d} " + " ".join(f"{c[x]:6d}" for x in
              ("valu", "vmov", "salu", "lds", "s_nop", "spill_lane", "agpr_move")))
    print(f"{'(all marked sections)':28s} {sum(tot.values()) - tot['wait']:6d}")
    print("marks in layout order:", len(order))


if __name__ == "__main__":
    main()
