"""Packaging (reference ``/root/reference/setup.py``).

``pip install -e .`` (or ``python setup.py build_ext --inplace``) compiles the gfx950 extension
in-tree through ``build_ext.py`` -- explicit ``hipcc --offload-arch=gfx950`` objects linked
against torch's HIP runtime -- so the ``_C.so`` lives next to the Python package.  Hydra is not
a dependency: the run config loader reads the same YAML with ``pyyaml``.
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext as _build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class HipBuild(_build_ext):
    """Delegate to build_ext.build(): one hipcc object per kernel file, incremental."""

    def run(self):
        sys.path.insert(0, ROOT)
        import build_ext as hb

        hb.build(jobs=os.cpu_count() or 4)


setup(
    name="mingpt-distributed-amd",
    version="0.1.0",
    description="MI355X-native GPT training and inference: gfx950 HIP kernels + RCCL data parallelism",
    license="MIT",
    packages=find_packages(include=["mingpt_distributed_amd", "mingpt_distributed_amd.*"]),
    package_data={"mingpt_distributed_amd": ["_C*.so"]},
    python_requires=">=3.9",
    install_requires=["torch", "pyyaml", "fsspec", "numpy"],
    extras_require={"s3": ["boto3", "s3fs"], "hf": ["safetensors"]},
    cmdclass={"build_ext": HipBuild},
    entry_points={"console_scripts": ["mingpt-train=mingpt_distributed_amd.train:main"]},
)
