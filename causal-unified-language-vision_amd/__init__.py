"""cullavo_amd: MI355X (gfx950)-native CuLLaVO forward/backward hot path.

Hand-written HIP kernels (libcullavo_hip.so, C-ABI in include/cullavo_capi.h) wrapped as
PyTorch-ROCm autograd Functions behind the reference's module API
(reference cullavo/arch_cullavo.py CuLLaVOModel, modeling/architectures/cullavo_model.py,
pipeline/CuLLaVOPipeline.py, trainer/cullavo_trainer.py).
"""
__version__ = "0.1.0"


def build(force: bool = False, verbose: bool = False) -> str:
    from .build import build as _b

    return _b(force=force, verbose=verbose)
