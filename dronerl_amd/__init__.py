"""dronerl_amd — MI355X-native batched DroneRL environment step.

The hot path of nyx-ai/droneRL (env reset / step / windowed observation) as
hand-written HIP kernels for gfx950 behind a C ABI (include/dronerl.h,
libdronerl.so), with two Python façades:

  dronerl_amd.BatchedDeliveryDrones   batched, jax_impl-shaped API on torch tensors
  dronerl_amd.compat                  torch_impl dict API drop-in (DeliveryDrones,
                                      WindowedGridView, set_seed)

Semantics are torch_impl's, bit-exact.  See DESIGN.md and INTEGRATION.md.
"""
from .constants import Action, Object
from .params import EnvParams, side_from_density

__all__ = ["Action", "Object", "EnvParams", "side_from_density", "BatchedDeliveryDrones", "DroneEnvState"]


def __getattr__(name):
    # torch-dependent pieces load lazily so `import dronerl_amd` stays light
    if name in ("BatchedDeliveryDrones", "DroneEnvState"):
        from . import env
        return getattr(env, name)
    raise AttributeError(name)
