"""Build the in-tree HIP extension for gfx950:  python setup.py build_ext --inplace

The CDNA4 kernels (``sheeprl_prey_amd/ops/csrc/*.hip``) are compiled directly by ``hipcc
--offload-arch=gfx950`` into objects (no hipify pass: the sources are HIP already); the torch
bindings (``bindings.cpp``) are a host-only C++ extension linked against them.  The .so lands
next to its Python package (``sheeprl_prey_amd/ops/_C*.so``) so it travels with the source tree;
nothing is installed into site-packages.
"""
import glob
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join("sheeprl_prey_amd", "ops", "csrc")
ARCH = os.environ.get("SRL_OFFLOAD_ARCH", "gfx950")
HIPCC_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=fast-honor-pragmas", "-munsafe-fp-atomics",
               "-Wno-unused-result"]

ext_modules = []
cmdclass = {}
try:
    from torch.utils.cpp_extension import BuildExtension, CppExtension

    class HipBuildExt(BuildExtension):
        """Compile every ``.hip`` translation unit with hipcc (in parallel, only when stale), then
        link them into the bindings extension."""

        def build_extensions(self):
            hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
            obj_dir = os.path.join(self.build_temp, "hip_objs")
            os.makedirs(obj_dir, exist_ok=True)
            srcs = sorted(glob.glob(os.path.join(HERE, CSRC, "*.hip")))
            headers = glob.glob(os.path.join(HERE, CSRC, "*.h"))
            newest_header = max((os.path.getmtime(h) for h in headers), default=0.0)

            def compile_one(src):
                obj = os.path.join(obj_dir, os.path.basename(src)[:-4] + ".o")
                if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_header):
                    return obj
                cmd = [hipcc, "-c", src, "-o", obj, "-I", os.path.join(HERE, CSRC)] + HIPCC_FLAGS
                print(" ".join(cmd), flush=True)
                subprocess.check_call(cmd)
                return obj

            jobs = int(os.environ.get("MAX_JOBS", "8"))
            with ThreadPoolExecutor(max_workers=max(1, jobs)) as pool:
                objs = list(pool.map(compile_one, srcs))
            for ext in self.extensions:
                ext.extra_objects = list(ext.extra_objects or []) + objs
            super().build_extensions()

    ext_modules.append(
        CppExtension(
            name="sheeprl_prey_amd.ops._C",
            sources=[os.path.join(CSRC, "bindings.cpp"), os.path.join(CSRC, "conv_bindings.cpp"),
                     os.path.join(CSRC, "ext_bindings.cpp"), os.path.join(CSRC, "sac_bindings.cpp")],
            include_dirs=[os.path.join(HERE, CSRC), os.path.join(ROCM, "include")],
            library_dirs=[os.path.join(ROCM, "lib")],
            libraries=["amdhip64", "c10_hip", "torch_hip"],
            define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
            extra_compile_args=["-O3", "-std=c++17"],
        )
    )
    cmdclass["build_ext"] = HipBuildExt.with_options(use_ninja=True)
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
