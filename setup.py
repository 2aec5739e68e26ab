"""Build the in-tree HIP extension for gfx950:  python setup.py build_ext --inplace

The .so lands next to its Python package (sheeprl_prey_amd/ops/_C*.so) so it travels with
the source tree; nothing is installed into site-packages.
"""
import glob
import os

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

ext_modules = []
cmdclass = {}
try:
    from torch.utils.cpp_extension import BuildExtension, CUDAExtension

    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join("sheeprl_prey_amd", "ops", "csrc")
    sources = sorted(glob.glob(os.path.join(csrc, "*.hip"))) + [os.path.join(csrc, "bindings.cpp")]
    ext_modules.append(
        CUDAExtension(
            name="sheeprl_prey_amd.ops._C",
            sources=sources,
            include_dirs=[os.path.join(here, csrc)],
            extra_compile_args={
                "cxx": ["-O3", "-std=c++17"],
                "nvcc": ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast", "-munsafe-fp-atomics"],
            },
        )
    )
    cmdclass["build_ext"] = BuildExtension.with_options(use_ninja=True)
except Exception as e:  # pragma: no cover
    print("HIP extension disabled:", e)

setup(
    name="sheeprl_prey_amd",
    version="0.1.0",
    packages=find_packages(include=["sheeprl_prey_amd", "sheeprl_prey_amd.*"]),
    package_data={"sheeprl_prey_amd": ["configs/**/*.yaml", "configs/*.yaml", "ops/csrc/*"]},
    ext_modules=ext_modules,
    cmdclass=cmdclass,
    entry_points={"console_scripts": ["sheeprl=sheeprl_prey_amd.cli:run", "sheeprl-eval=sheeprl_prey_amd.cli:evaluation"]},
)
