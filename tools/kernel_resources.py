#!/usr/bin/env python3
"""Per-kernel resources of the built library (lib/libgsplat.so): the gfx950 code object is
unbundled from .hip_fatbin and its metadata notes read (VGPRs, SGPRs, LDS, scratch bytes).

    python tools/kernel_resources.py [path/to/libgsplat.so]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def demangle_short(name):
    """k_name<template args> (llvm-cxxfilt; the namespaces and the parameter list dropped)."""
    try:
        d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        d = re.sub(r"\([^()]*\)$", "", d.replace("(anonymous namespace)::", "").replace("gs::", ""))
        d = re.sub(r"^void ", "", d)
        if d.startswith("k_"):
            return d.replace(" ", "")
    except OSError:
        pass
    m = re.search(r"(k_[a-z0-9_]+)E?(I[^E]*E)?", name)
    if not m:
        return name
    base = m.group(1)
    if "ILb1E" in name:
        base += "<true>"
    elif "ILb0E" in name:
        base += "<false>"
    elif "ILi8EE" in name:
        base += "<8>"
    return base


def kernel_resources(lib):
    """{kernel: {"vgpr": n, "sgpr": n, "lds": bytes, "scratch": bytes}} from the library's code object."""
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "co.elf")
        # an explicit output file: objcopy with one file argument rewrites it in place, which
        # corrupts any process that has the library mapped
        subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, lib, os.path.join(td, "copy.so")],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True,
                       capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        s = line.strip()
        if s.startswith("- .agpr_count:") or s.startswith(".agpr_count:"):
            cur = {}
        m = re.match(r"-?\s*\.(\w+):\s+(\S+)", s)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "name":
            cur["name"] = v
            out[demangle_short(v)] = cur
        elif k in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size"):
            cur[{"vgpr_count": "vgpr", "sgpr_count": "sgpr", "group_segment_fixed_size": "lds",
                 "private_segment_fixed_size": "scratch"}[k]] = int(v)
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gaussian-splatting-web_amd", "lib", "libgsplat.so")
    res = kernel_resources(lib)
    print("%-24s %6s %6s %8s %8s" % ("kernel", "vgpr", "sgpr", "lds", "scratch"))
    for k in sorted(res):
        r = res[k]
        print("%-24s %6d %6d %8d %8d" % (k, r.get("vgpr", -1), r.get("sgpr", -1), r.get("lds", -1), r.get("scratch", -1)))


if __name__ == "__main__":
    main()
