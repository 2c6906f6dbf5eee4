"""Resolve the addresses of a failure-handler stack trace ("@ 0x7f..." lines, as rocprofv3's
glog handler prints them) against a /proc/<pid>/maps copy of the same process
(scripts/refprof_repro.py writes one), then name the function with llvm-symbolizer on the
library file (the GPU box runs this same image, so the files are identical here).

    python scripts/symbolize_trace.py gpurun_out/x.log gpurun_out/repro_maps.txt
"""
import re
import subprocess
import sys

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    out = []
    for line in open(path):
        f = line.split()
        if len(f) < 5:
            continue
        lo, hi = (int(x, 16) for x in f[0].split("-"))
        out.append((lo, hi, f[1], int(f[2], 16), f[5] if len(f) > 5 else ""))
    return out


def where(maps, a):
    for lo, hi, perm, off, name in maps:
        if lo <= a < hi:
            return lo, hi, perm, off, name
    return None


def main():
    log, mp = sys.argv[1], sys.argv[2]
    maps = load_maps(mp)
    addrs = []
    for line in open(log):
        m = re.search(r"SIGSEGV \(@(0x[0-9a-f]+)\)", line)
        if m:
            addrs.append(("fault address", int(m.group(1), 16)))
        m = re.search(r"PC: @\s+(0x[0-9a-f]+)", line)
        if m:
            addrs.append(("faulting PC", int(m.group(1), 16)))
        m = re.match(r"\s+@\s+(0x[0-9a-f]+)\s*(.*)", line)
        if m:
            addrs.append((m.group(2) or "frame", int(m.group(1), 16)))
    for label, a in addrs:
        w = where(maps, a)
        if w is None:
            # the nearest mappings on either side (an address in no mapping: unmapped memory)
            below = max((x for x in maps if x[1] <= a), key=lambda x: x[1], default=None)
            above = min((x for x in maps if x[0] > a), key=lambda x: x[0], default=None)
            print("%-28s %#x  UNMAPPED; below: %s, above: %s" % (
                label, a,
                below and "%#x-%#x %s %s" % (below[0], below[1], below[2], below[4]),
                above and "%#x-%#x %s %s" % (above[0], above[1], above[2], above[4])))
            continue
        lo, hi, perm, off, name = w
        foff = a - lo + off
        fn = ""
        if name.startswith("/") and "x" in perm:
            try:
                r = subprocess.run([SYM, "--obj=" + name, "--functions=short", hex(foff)],
                                   capture_output=True, text=True, timeout=30)
                fn = r.stdout.split("\n")[0]
            except Exception as e:      # noqa: BLE001
                fn = "(%s)" % e
        print("%-28s %#x  %s+%#x [%s %#x-%#x] %s" % (label, a, name or "[anon]", foff, perm, lo, hi, fn))


if __name__ == "__main__":
    main()
