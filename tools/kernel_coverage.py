#!/usr/bin/env python3
"""Which kernels of libpwc_hotpath.so a run touched: the .so's kernel symbols (nm -C) against the
kernel names in a rocprofv3 --kernel-trace --stats CSV (e.g. the -m gpu suite under the tracer).

    python tools/kernel_coverage.py <run_kernel_stats.csv> [libpwc_hotpath.so] > report.txt
"""
import csv
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def so_kernels(path):
    out = subprocess.run(["nm", "-C", path], capture_output=True, text=True, check=True).stdout
    names = set()
    for line in out.splitlines():
        parts = line.split(" ", 2)
        if len(parts) < 3 or parts[1] not in "BbDdRrVvWw" or "(" not in parts[2]:
            continue
        name = parts[2]
        if name.startswith("void "):
            name = name[5:]
        if name.startswith("pwc::") and not re.search(r"attr|guard|spec|::g_|lds_limit", name):
            names.add(name)
    return names


def base(name):
    """kernel name without the argument list (template arguments kept)."""
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def family(name):
    return re.sub(r"<.*", "", base(name))


def main():
    stats = sys.argv[1]
    so = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        ROOT, "pwc-net_pytorch_amd", "pwcnet_amd", "lib", "libpwc_hotpath.so")
    hit = set()
    for r in csv.DictReader(open(stats)):
        n = r["Name"]
        if n.startswith("void "):
            n = n[5:]
        hit.add(base(n))
    kernels = sorted(so_kernels(so), key=base)
    fams = {}
    for k in kernels:
        fams.setdefault(family(k), []).append(base(k) in hit)
    print(f"{sum(base(k) in hit for k in kernels)} of {len(kernels)} kernel instantiations hit; "
          f"{sum(any(v) for v in fams.values())} of {len(fams)} families hit")
    for f, v in sorted(fams.items()):
        print(f"{'HIT ' if any(v) else 'MISS'} {f}: {sum(v)}/{len(v)} instantiations")
    print("# instantiations not hit:")
    for k in kernels:
        if base(k) not in hit:
            print("  " + base(k))


if __name__ == "__main__":
    main()
