"""Build the native extension ``mpi_pytorch_amd._C`` for gfx950 (MI355X) in-tree.

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

Sources: hand-written HIP kernels (``csrc/kernels/*.hip``), the C++ host runtime
(``csrc/runtime``) and the torch binding layer (``csrc/bindings.cpp``).  hipcc
cross-compiles for gfx950 without a GPU present.
"""
import glob
import os

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

from setuptools import setup  # noqa: E402
from torch.utils.cpp_extension import BuildExtension, CUDAExtension  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
kernels = sorted(glob.glob(os.path.join("csrc", "kernels", "*.hip")))
sources = [os.path.join("csrc", "bindings.cpp"), os.path.join("csrc", "runtime", "runtime.cpp")]
sources += kernels

ext = CUDAExtension(
    name="mpi_pytorch_amd._C",
    sources=sources,
    include_dirs=[os.path.join(ROOT, "csrc")],
    extra_compile_args={
        "cxx": ["-O3", "-std=c++17"],
        "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=fast"],
    },
    libraries=["rocprofiler-sdk-roctx"],
    library_dirs=["/opt/rocm/lib"],
)

setup(
    name="mpi_pytorch_amd",
    version="0.1.0",
    packages=["mpi_pytorch_amd"],
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
