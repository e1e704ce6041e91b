"""Build script for arena_amd's native components (in-tree).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

builds ``arena_amd/_C*.so`` (HIP kernels + torch bindings, gfx950 only). The C++ runtime tools
(supervisor, GPU probe) are built by ``arena_amd/_build.py`` with plain g++ (no GPU needed).
"""
import os

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

ext_modules = []
cmdclass = {}
try:
    from torch.utils.cpp_extension import BuildExtension, CUDAExtension

    here = os.path.dirname(os.path.abspath(__file__))
    ext_modules = [
        CUDAExtension(
            "arena_amd._C",
            sources=["csrc/ops/bindings.cpp", "csrc/ops/mlp_kernels.hip"],
            include_dirs=[os.path.join(here, "csrc", "ops")],
            extra_compile_args={
                "cxx": ["-O3", "-std=c++17"],
                "nvcc": ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast"],
            },
        )
    ]
    cmdclass = {"build_ext": BuildExtension.with_options(use_ninja=True)}
except ImportError:  # pragma: no cover - torch is always present in this image
    pass

setup(
    name="arena_amd",
    version=open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "VERSION")).read().strip(),
    packages=find_packages(include=["arena_amd", "arena_amd.*"]),
    ext_modules=ext_modules,
    cmdclass=cmdclass,
    entry_points={"console_scripts": ["arena=arena_amd.cli.main:main",
                                      "arena-jobmon=arena_amd.runtime.jobmon:main"]},
)
