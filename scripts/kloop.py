"""Register report of one kernel in a hipcc -S device assembly: VGPR / SGPR spills and, for every
loop of 150..1300 instructions, its size, scratch accesses and SGPR-lane spill moves.
    python scripts/kloop.py /tmp/chain.s chain_kernelILi5ELi8ELi2ELi8
"""
import re
import sys


def main(path, pat):
    src = open(path).read()
    m = re.search(r"^(_Z\w*%s\w*):" % pat, src, re.M)
    name = m.group(1)
    body = src[m.start():src.index(".Lfunc_end", m.start())].split("\n")
    meta = src[src.index(".name:           " + name):][:1200]
    for key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
        print("%s: %s" % (key, re.search(r"\.%s:\s+(\d+)" % key, meta).group(1)))
    labels = {re.match(r"^(\.LBB\d+_\d+):", l).group(1): i for i, l in enumerate(body)
              if re.match(r"^\.LBB\d+_\d+:", l)}
    seen = set()
    for i, l in enumerate(body):
        mm = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if mm and labels.get(mm.group(2), 1 << 30) < i:
            a = labels[mm.group(2)]
            blk = body[a:i]
            n = sum(1 for x in blk if re.match(r"^\s+[vsdgb]", x))
            if 150 < n < 1300 and a not in seen and len(seen) < 8:
                seen.add(a)
                print("loop @%d: %d instrs, scratch %d, sgpr-lane %d" % (
                    a, n, sum("scratch_" in x for x in blk),
                    sum(("v_readlane_b32 s" in x) or ("v_writelane" in x) for x in blk)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "chain_kernelILi5ELi8ELi2ELi8")
