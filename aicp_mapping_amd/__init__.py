"""aicp_mapping_amd — MI355X-native ICP registration core for AICP (zbqq/aicp_mapping).

The product is libaicp_hip.so (C-ABI in include/aicp_hip.h, HIP kernels for gfx950 under
csrc/). This package mirrors the reference's registrator / overlapper plugin interfaces on top
of it (registration.py) and ships the seeded synthetic scenes of the benchmark (synthetic.py).
Importing `aicp_mapping_amd.registration` or `aicp_mapping_amd._lib` loads the HIP library and
fails loudly if it is missing.
"""

__all__ = ["registration", "synthetic"]


def __getattr__(name):
    if name in ("registration", "_lib", "synthetic"):
        import importlib

        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
