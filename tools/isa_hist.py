"""Instruction histogram of a line range of a gfx950 assembly listing
(hipcc --cuda-device-only -S).  Diagnostic only.

    python tools/isa_hist.py listing.s [first_line last_line]
"""
import collections
import sys


def main():
    lines = open(sys.argv[1]).read().splitlines()
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else len(lines)
    cnt = collections.Counter()
    for ln in lines[lo - 1:hi]:
        t = ln.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        cnt[t.split()[0]] += 1
    for op, n in cnt.most_common(28):
        print(f"{n:6d} {op}")
    print(f"total {sum(cnt.values())}")


if __name__ == "__main__":
    main()
