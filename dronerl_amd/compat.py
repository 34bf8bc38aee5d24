"""Drop-in for torch_impl's dict API (single env), backed by the HIP kernels.

Mirrors /root/reference torch_impl/env/env.py (``Drone`` :8-15,
``DeliveryDrones`` :18-310) and torch_impl/env/wrappers.py
(``GridView`` :34-43, ``WindowedGridView`` :46-73) so evaluator-style callers
(drone_evaluator.py:106-162, train_torch.py:41-120) can switch imports:

    from dronerl_amd.compat import DeliveryDrones, WindowedGridView

Like the reference, the env draws from Python's *global* ``random`` stream:
before each reset/step the stream's state (``random.getstate()``) is loaded
into the env's device MT19937 row, and after it the advanced state is written
back with ``random.setstate()``.  ``set_seed(env, s); env.reset()`` therefore
reproduces the reference bit for bit.  Every step runs on the GPU
(drl_step + drl_obs); only the RNG words and the resulting state cross PCIe.

Differences (documented, deliberate): env_params is copied, not an alias of the
class-level DEFAULT_CONFIG (the reference's env.py:54-55 leaks params across
instances).
"""
from __future__ import annotations

import random

import numpy as np
import torch

from .constants import Object
from .env import BatchedDeliveryDrones
from .params import TORCH_DEFAULT_CONFIG, EnvParams

_OBJ_DICTS = (("skyscrapers", Object.SKYSCRAPER), ("stations", Object.STATION), ("dropzones", Object.DROPZONE),
              ("packets", Object.PACKET))


class Discrete:
    """gym.spaces.Discrete surface used by the reference (env.py:53; seeding
    and sampling as gym 0.25.2: PCG64 over SeedSequence)."""

    def __init__(self, n: int, start: int = 0):
        self.n, self.start = int(n), int(start)
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))

    def seed(self, seed=None):
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return [seed]

    def sample(self) -> int:
        return int(self.start + self.np_random.integers(self.n))

    def contains(self, x) -> bool:
        return isinstance(x, (int, np.integer)) and self.start <= int(x) < self.start + self.n


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype


class Drone:
    """env.py:8-15."""

    def __init__(self, index):
        self.index = index
        self.packet = False
        self.charge = 100

    def __repr__(self):
        return f'D{self.index}, packet={self.packet}, charge={self.charge}'


class DeliveryDrones:
    """torch_impl DeliveryDrones (env.py:18) on one GPU env."""

    ACTION_TO_DIRECTION = [(0, -1), (1, 0), (0, 1), (-1, 0), (0, 0)]
    NUM_ACTIONS = len(ACTION_TO_DIRECTION)
    DEFAULT_CONFIG = dict(TORCH_DEFAULT_CONFIG)
    metadata = {'render.modes': ['ansi']}

    def __init__(self, env_params={}, device=None):
        self.action_space = Discrete(self.NUM_ACTIONS)
        self.env_params = dict(self.DEFAULT_CONFIG)
        self.env_params.update(env_params)
        self._device = device
        self._gpu = None
        self._gpu_key = None
        self._drone_objs = {}
        self.reset()

    @property
    def drones_list(self):
        return list(self.drones.values())

    # --------------------------------------------------------------- core --
    def _ensure_gpu(self):
        p = EnvParams.from_torch_config(self.env_params)
        key = (p.side, p.n_drones, p.charge, p.discharge, p.packets_factor, p.dropzones_factor, p.stations_factor,
               p.skyscrapers_factor, p.pickup_reward, p.delivery_reward, p.crash_reward, p.charge_reward)
        if self._gpu is None or key != self._gpu_key:
            self._gpu = BatchedDeliveryDrones(p, 1, device=self._device)
            self._gpu_key = key
            self._drone_objs = {i: Drone(i) for i in range(p.n_drones)}
        return self._gpu

    def _push_rng(self):
        st = random.getstate()
        self._gpu.set_mt_words(list(st[1]))

    def _pull_rng(self):
        w = self._gpu.mt_words()[0].tolist()
        st = random.getstate()
        random.setstate((st[0], tuple(int(v) for v in w), st[2]))

    def _sync_host(self):
        g = self._gpu
        d = g.decode()
        ground = d["ground"][0].cpu().numpy()
        order = d["order"][0].cpu().tolist()
        ys, xs = d["y"][0].cpu().tolist(), d["x"][0].cpu().tolist()
        ch, car = d["charge"][0].cpu().tolist(), d["carrying"][0].cpu().tolist()
        self.drones = {}
        for i in order:
            dr = self._drone_objs[i]
            dr.charge = int(ch[i])
            dr.packet = bool(car[i])
            self.drones[(ys[i], xs[i])] = dr
        for name, code in _OBJ_DICTS:
            yy, xx = np.nonzero(ground == int(code))
            setattr(self, name, {(int(a), int(b)): True for a, b in zip(yy, xx)})

    def reset(self, seed=0):
        """env.py:68-101 (``seed`` is ignored, as in the reference)."""
        g = self._ensure_gpu()
        self.n_drones = self.env_params['n_drones']
        self.side_size = g.side
        self.shape = (self.side_size, self.side_size)
        for dr in self._drone_objs.values():
            dr.charge, dr.packet = 100, False
        self._push_rng()
        g.reset(seed=None)
        self._pull_rng()
        self._sync_host()
        return self.get_state(), None

    def get_state(self):
        return {
            'drones': self.drones,
            'stations': self.stations,
            'dropzones': self.dropzones,
            'packets': self.packets,
            'skyscrapers': self.skyscrapers,
        }

    def _actions_tensor(self, actions: dict):
        N = self.n_drones
        a = np.zeros(N, dtype=np.int32)
        for i in range(N):
            v = int(actions[i])  # KeyError for a missing drone, as env.py:125
            if not -self.NUM_ACTIONS <= v < self.NUM_ACTIONS:
                raise IndexError("list index out of range")
            a[i] = v
        return torch.from_numpy(a).reshape(1, N)

    def step(self, actions):
        """env.py:112-215.  Returns (state, rewards, dones, None, info)."""
        g = self._gpu
        a = self._actions_tensor(actions)
        self._push_rng()
        r, d = g.step(a)
        self._pull_rng()
        self._sync_host()
        r = r[0].cpu().tolist()
        d = d[0].cpu().tolist()
        rewards = {index: _py_reward(r[index], self.env_params) for index in actions.keys()}
        dones = {index: bool(d[index]) for index in actions.keys()}
        return self.get_state(), rewards, dones, None, {}

    def _window_obs(self, radius: int) -> dict:
        """WindowedGridView windows for every drone, {index: float64 [W,W,6]} in dict order."""
        g = self._gpu
        if radius != g.params.window_radius:
            self._gpu = BatchedDeliveryDrones(g.params.replace(window_radius=radius), 1, device=self._device)
            self._gpu.state = g.state
            g = self._gpu
        o = g.get_obs().cpu().numpy()[0].astype(np.float64)
        return {drone.index: o[drone.index].copy() for drone in self.drones.values()}

    def _grid_obs(self) -> dict:
        """GridView grids for every drone, {index: float32 [G,G,6]} in dict order."""
        grid = self._gpu.get_grid().cpu().numpy()[0]
        return {drone.index: grid.copy() for drone in self.drones.values()}

    # ------------------------------------------------------------ helpers --
    def render(self, mode='ansi'):
        return self.__str__()

    def format_actions(self, actions: dict):
        return {d: ['←', '↓', '→', '↑', 'X'][i] for d, i in actions.items()}

    def __str__(self):
        lines = ["_" * self.shape[0] * 2]
        for y in range(self.shape[0]):
            line_str = ''
            for x in range(self.shape[1]):
                p = (y, x)
                if p in self.drones:
                    t = f'{self.drones[p].index}'
                elif p in self.packets:
                    t = 'x'
                elif p in self.dropzones:
                    t = 'D'
                elif p in self.stations:
                    t = '@'
                elif p in self.skyscrapers:
                    t = '#'
                else:
                    t = '.'
                line_str += t.ljust(2)
            lines.append(line_str)
        lines.append("_" * self.shape[0] * 2)
        return '\n'.join(lines)


def _py_reward(v: float, params: dict):
    """Map the kernel's f32 reward back to the exact Python value the reference
    returns (one of the configured rewards, or 0)."""
    for k in ('crash_reward', 'charge_reward', 'pickup_reward', 'delivery_reward'):
        ref = params[k]
        if np.float32(ref) == np.float32(v):
            return ref
    return 0 if v == 0 else v


class WindowedGridView:
    """torch_impl WindowedGridView (wrappers.py:46-73) over a compat env."""

    def __init__(self, env: DeliveryDrones, radius: int):
        assert radius > 0, "Radius should be strictly positive"
        self.env = env
        self.radius = radius
        self.observation_space = Box(0, 1, shape=(radius * 2 + 1, radius * 2 + 1, 6), dtype=float)

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def action_space(self):
        return self.env.action_space

    def observation(self, _):
        return self.env._window_obs(self.radius)

    def reset(self, **kw):
        self.env.reset(**kw)
        return self.observation(None)

    def step(self, actions):
        _, r, d, trunc, info = self.env.step(actions)
        return self.observation(None), r, d, trunc, info

    def render(self, mode='ansi'):
        return self.env.render(mode)


class GridView(WindowedGridView):
    """torch_impl GridView (wrappers.py:34-43): every drone sees the whole
    [side, side, 6] float32 grid (no wall padding)."""

    def __init__(self, env: DeliveryDrones):
        self.env = env
        self.observation_space = Box(0, 1, shape=(env.side_size, env.side_size, 6), dtype=float)

    def observation(self, _):
        return self.env._grid_obs()


def set_seed(env, seed):
    """torch_impl/helpers/rl_helpers.py:12-18 (env/action-space/numpy/torch/random)."""
    env.reset(seed=seed)
    env.action_space.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    random.seed(seed)
