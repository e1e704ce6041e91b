#!/usr/bin/env python3
"""Register / LDS / scratch report of the gfx950 kernels in a built HIP object (no GPU needed).

    python tools/kernel_regs.py build/hip_objs/conv_kernels.o [name-substring ...]

Extracts the object's offload bundle (``.hip_fatbin`` -> ``clang-offload-bundler``), reads the
code object's AMDGPU metadata note (``llvm-readelf --notes``) and prints one line per kernel:
VGPRs, AGPRs, SGPRs, spilled VGPRs/SGPRs, private (scratch) bytes, static LDS bytes and the
demangled name. A kernel that spills or uses scratch is flagged with ``!``: on the occupancy-
bound conv tiles a spill shows up as a few % of kernel time (docs/perf.md).
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import yaml

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")


def _run(*args) -> str:
    return subprocess.run(list(args), check=True, capture_output=True, text=True).stdout


def kernels(obj: str):
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "k.co")
        _run(os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj,
             os.path.join(td, "dummy.o"))
        _run(os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
             f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}")
        notes = _run(os.path.join(LLVM, "llvm-readelf"), "--notes", co)
    start = notes.index("---")
    end = notes.index("...", start)
    meta = yaml.safe_load(notes[start:end])
    names = [k[".name"] for k in meta["amdhsa.kernels"]]
    dem = subprocess.run(["c++filt"], input="\n".join(names), check=True, capture_output=True,
                         text=True).stdout.splitlines()
    for k, d in zip(meta["amdhsa.kernels"], dem):
        yield {"name": d, "vgpr": k.get(".vgpr_count"), "agpr": k.get(".agpr_count", 0),
               "sgpr": k.get(".sgpr_count"), "vspill": k.get(".vgpr_spill_count", 0),
               "sspill": k.get(".sgpr_spill_count", 0),
               "scratch": k.get(".private_segment_fixed_size", 0),
               "lds": k.get(".group_segment_fixed_size", 0)}


def main(argv):
    if not argv:
        print(__doc__)
        return 2
    obj, pats = argv[0], argv[1:]
    print(f"{'':1} {'vgpr':>4} {'agpr':>4} {'sgpr':>4} {'vsp':>4} {'ssp':>4} {'scr':>5} {'lds':>6}  kernel")
    for k in kernels(obj):
        if pats and not any(p in k["name"] for p in pats):
            continue
        bad = "!" if (k["vspill"] or k["sspill"] or k["scratch"]) else " "
        name = k["name"].replace("(anonymous namespace)::", "")
        print(f"{bad} {k['vgpr']:>4} {k['agpr']:>4} {k['sgpr']:>4} {k['vspill']:>4} "
              f"{k['sspill']:>4} {k['scratch']:>5} {k['lds']:>6}  {name[:150]}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
