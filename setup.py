"""Build script for arena_amd's native components (in-tree).

    python setup.py build_ext --inplace

builds ``arena_amd/_C*.so``: the HIP kernels (``csrc/ops/*.hip``) are compiled by ``hipcc
--offload-arch=gfx950`` straight from source (no hipify pass, no CUDA sources anywhere) and linked
with the host-only torch binding TU. The C++ runtime tools (supervisor, GPU probe) are built by
``arena_amd/_build.py`` with plain g++ (no GPU needed).
"""
import os
import subprocess
import sys

from setuptools import find_packages, setup

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
if ARCH != "gfx950":
    raise SystemExit(f"arena_amd targets MI355X only (gfx950); PYTORCH_ROCM_ARCH={ARCH}")

HIP_SOURCES = ["csrc/ops/mlp_kernels.hip", "csrc/ops/bn_kernels.hip", "csrc/ops/pool_kernels.hip",
               "csrc/ops/conv_kernels.hip",
               "csrc/ccl/xgmi_ccl.hip"]
# ARENA_TIMELINE=1: instrumented build for tools/timeline.py (never the default)
TIMELINE = ["-DARENA_TIMELINE"] if os.environ.get("ARENA_TIMELINE") == "1" else []
if TIMELINE:  # ARENA_EXP ablation switches, instrumented builds only (see tools/timeline.py)
    TIMELINE += os.environ.get("ARENA_EXP_FLAGS", "").split()
CPP_SOURCES = ["csrc/ops/bindings.cpp"]

ext_modules = []
cmdclass = {}
try:
    from torch.utils.cpp_extension import BuildExtension, CppExtension

    sys.path.insert(0, os.path.join(HERE, "arena_amd", "ops"))
    from _srchash import source_hash  # noqa: E402

    src_hash = source_hash(os.path.join(HERE, "csrc", "ops"), os.path.join(HERE, "csrc", "ccl"))
    obj_dir = os.path.join(HERE, "build", "hip_objs")
    hip_objs = [os.path.join(obj_dir, os.path.basename(s).replace(".hip", ".o"))
                for s in HIP_SOURCES]

    class HipBuildExt(BuildExtension):
        """Compile .hip kernels with hipcc for gfx950, then link them into the torch extension."""

        def build_extensions(self):
            os.makedirs(obj_dir, exist_ok=True)
            hipcc = os.path.join(ROCM, "bin", "hipcc")
            cmds = []
            for src, obj in zip(HIP_SOURCES, hip_objs):
                srcp = os.path.join(HERE, src)
                deps = [srcp] + [os.path.join(HERE, "csrc", "ops", h)
                                for h in ("abi.h", "common.h", "adam.h")]
                if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d)
                                               for d in deps):
                    continue
                cmds.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                             "-ffp-contract=fast", "-I", os.path.join(HERE, "csrc", "ops"), "-c",
                             srcp, "-o", obj] + TIMELINE)
            # independent translation units: compile them concurrently (the conv kernels alone
            # take minutes; the others finish under it)
            from concurrent.futures import ThreadPoolExecutor
            jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
            for cmd in cmds:
                print(" ".join(cmd), flush=True)
            with ThreadPoolExecutor(jobs) as pool:
                for r in pool.map(lambda c: subprocess.run(c, check=True), cmds):
                    pass
            super().build_extensions()

    ext_modules = [
        CppExtension(
            "arena_amd._C",
            sources=CPP_SOURCES,
            include_dirs=[os.path.join(HERE, "csrc", "ops"), os.path.join(ROCM, "include")],
            extra_objects=hip_objs,
            library_dirs=[os.path.join(ROCM, "lib")],
            libraries=["amdhip64", "c10_hip", "torch_hip"],
            define_macros=[("ARENA_SRC_HASH", f'"{src_hash}"'), ("__HIP_PLATFORM_AMD__", "1"),
                           ("USE_ROCM", "1")],
            extra_compile_args=["-O3", "-std=c++17"] + TIMELINE,
        )
    ]
    cmdclass = {"build_ext": HipBuildExt.with_options(use_ninja=True)}
except ImportError:  # pragma: no cover - torch is always present in this image
    pass

setup(
    name="arena_amd",
    version=open(os.path.join(HERE, "VERSION")).read().strip(),
    packages=find_packages(include=["arena_amd", "arena_amd.*"]),
    ext_modules=ext_modules,
    cmdclass=cmdclass,
    entry_points={"console_scripts": ["arena=arena_amd.cli.main:main",
                                      "arena-jobmon=arena_amd.runtime.jobmon:main"]},
)
