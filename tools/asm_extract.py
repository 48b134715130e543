#!/usr/bin/env python3
"""Extract one kernel's body from a hipcc -S listing and summarise it per basic block.
Usage: python tools/asm_extract.py <file.s> <mangled-substring> [--dump]"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{pat}\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    if "--dump" in sys.argv:
        print("\n".join(body))
        return
    blk, n, kinds = body[0], 0, {}
    out = []
    for l in body[1:]:
        if re.match(r"^\.LBB\S*:", l):
            out.append((blk, n, kinds))
            blk, n, kinds = l.split(";")[0], 0, {}
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        n += 1
        k = op.split("_")[0] + "_" + (op.split("_")[1] if "_" in op else "")
        kinds[k] = kinds.get(k, 0) + 1
    out.append((blk, n, kinds))
    tot = sum(o[1] for o in out)
    print(f"{len(out)} blocks, {tot} instructions")
    for b, n, k in out:
        top = sorted(k.items(), key=lambda x: -x[1])[:6]
        print(f"{b[:40]:40s} {n:5d}  " + " ".join(f"{a}:{c}" for a, c in top))


if __name__ == "__main__":
    main()
