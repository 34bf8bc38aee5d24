"""Environment parameters.

Mirrors torch_impl ``DeliveryDrones.DEFAULT_CONFIG`` (env.py:28-42) and jax
``DroneEnvParams`` (jax_impl/env/env.py:11-26).  The grid side is either given
(jax ``grid_size``) or derived from ``drone_density`` exactly as torch_impl does
(``ceil(sqrt(n_drones / drone_density))``, env.py:75).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, fields, replace
from typing import Optional

from ._native import DrlLayout, DrlParams, check_value, lib

TORCH_DEFAULT_CONFIG = {
    'drone_density': 0.05,
    'n_drones': 3,
    'pickup_reward': 0,
    'delivery_reward': 1,
    'crash_reward': -1,
    'charge_reward': -0.1,
    'discharge': 10,
    'charge': 20,
    'packets_factor': 3,
    'dropzones_factor': 2,
    'stations_factor': 2,
    'skyscrapers_factor': 3,
    'rgb_render_rescale': 1.0,
}


def side_from_density(n_drones: int, drone_density: float) -> int:
    """env.py:75, in double precision."""
    return int(math.ceil(math.sqrt(n_drones / drone_density)))


@dataclass(frozen=True)
class EnvParams:
    n_drones: int = 3
    grid_size: Optional[int] = None
    drone_density: float = 0.05
    pickup_reward: float = 0.0
    delivery_reward: float = 1.0
    crash_reward: float = -1.0
    charge_reward: float = -0.1
    discharge: int = 10
    charge: int = 20
    packets_factor: int = 3
    dropzones_factor: int = 2
    stations_factor: int = 2
    skyscrapers_factor: int = 3
    window_radius: int = 3

    @property
    def side(self) -> int:
        if self.grid_size is not None:
            return int(self.grid_size)
        return side_from_density(self.n_drones, self.drone_density)

    @classmethod
    def from_torch_config(cls, cfg: dict, window_radius: int = 3) -> "EnvParams":
        """From a torch_impl env_params dict (missing keys take DEFAULT_CONFIG values)."""
        c = dict(TORCH_DEFAULT_CONFIG)
        c.update(cfg)
        known = {f.name for f in fields(cls)}
        kw = {k: v for k, v in c.items() if k in known}
        return cls(window_radius=window_radius, **kw)

    def replace(self, **kw) -> "EnvParams":
        return replace(self, **kw)

    def to_c(self) -> DrlParams:
        # The kernels do charge / factor arithmetic on integers (the reference
        # does it on Python numbers, env.py:79-82,152-155): refuse fractions
        # instead of truncating them.
        for name in ("charge", "discharge", "packets_factor", "dropzones_factor", "stations_factor",
                     "skyscrapers_factor", "n_drones", "window_radius"):
            v = getattr(self, name)
            if isinstance(v, bool) or float(v) != int(v):
                raise ValueError(f"{name}={v!r}: the C ABI supports integer values only")
        return DrlParams(self.side, self.n_drones, int(self.charge), int(self.discharge), int(self.packets_factor),
                         int(self.dropzones_factor), int(self.stations_factor), int(self.skyscrapers_factor),
                         int(self.window_radius), float(self.pickup_reward), float(self.delivery_reward),
                         float(self.crash_reward), float(self.charge_reward))

    def layout(self) -> DrlLayout:
        L = DrlLayout()
        import ctypes
        check_value(lib().drl_layout_query(ctypes.byref(self.to_c()), ctypes.byref(L)))
        return L

    def as_dict(self) -> dict:
        return asdict(self)
