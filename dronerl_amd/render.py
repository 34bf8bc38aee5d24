"""State decode for rendering.

torch_impl/render_util.py:37-59 convert_for_rendering(env) and
jax_impl/render_util.py:18-30 convert_jax_state: the arrays common/render.py's
Renderer.render_frame takes -- ground [side, side] (object code or None),
air [side, side] (drone index or None), carrying_package [N] and charge [N]
by drone index.  `from_arrays` is the core (decoded numpy state);
`convert_for_rendering` takes a compat env (as the evaluator calls it) and
`convert_batched` one env of a BatchedDeliveryDrones batch.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .constants import Object

_ORDER = (Object.DROPZONE, Object.STATION, Object.SKYSCRAPER, Object.PACKET)  # render_util.py:40-47 write order


def from_arrays(ground: np.ndarray, y, x, charge, carrying) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """ground u8 [G, G] codes; y/x/charge/carrying [N] by drone index."""
    G = ground.shape[0]
    g = np.full((G, G), None)
    for code in _ORDER:
        for yy, xx in zip(*np.nonzero(ground == int(code))):
            g[yy, xx] = code
    air = np.full((G, G), None)
    for i in range(len(y)):
        air[int(y[i]), int(x[i])] = i
    return g, air, np.array([bool(c) for c in carrying]), np.array([int(c) for c in charge])


def convert_for_rendering(env):
    """torch_impl/render_util.py:37-59 for a dronerl_amd.compat env (or wrapper)."""
    base = getattr(env, "env", env)
    G = base.side_size
    ground = np.zeros((G, G), np.uint8)
    for name, code in (("dropzones", Object.DROPZONE), ("stations", Object.STATION),
                       ("skyscrapers", Object.SKYSCRAPER), ("packets", Object.PACKET)):
        for (yy, xx) in getattr(base, name).keys():
            ground[yy, xx] = int(code)
    drones = sorted(base.drones.items(), key=lambda kv: kv[1].index)
    y = [p[0] for p, _ in drones]
    x = [p[1] for p, _ in drones]
    return from_arrays(ground, y, x, [d.charge for _, d in drones], [d.packet for _, d in drones])


def convert_batched(env, e: int):
    """The same arrays for env `e` of a BatchedDeliveryDrones batch (one device decode)."""
    d = env.decode()
    return from_arrays(d["ground"][e].cpu().numpy(), d["y"][e].cpu().numpy(), d["x"][e].cpu().numpy(),
                       d["charge"][e].cpu().numpy(), d["carrying"][e].cpu().numpy())
