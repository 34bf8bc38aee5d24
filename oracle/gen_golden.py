"""ORACLE TOOLING ONLY — generates tests/golden/* by importing the reference.

Runs in the build container only (it reads /root/reference, which does not
exist on the GPU box).  It imports /root/reference/torch_impl/env with the
gym stand-in in oracle/gymshim (the reference's only missing dependency,
torch_impl/requirements.txt:1 pins gym 0.25.2), drives it exactly as the
reference's own tests and drivers do -- ``random.seed(s); env.reset()``
(torch_impl/helpers/rl_helpers.py:12-18) then ``env.step({idx: action})``
(env.py:112) and ``WindowedGridView.observation`` (wrappers.py:55-73) -- and
writes plain data (inputs and outputs) as fixtures:

  tests/golden/ref_tests.npz    the reference's own golden tests as data:
                                test_windowedgridview.py, test_env_single_drone.py,
                                test_env_multiple_drones.py (incl. the gym-PCG64
                                sampled random actions those scripts use)
  tests/golden/traj_<name>.npz  seeded uniform-random-action trajectories per
                                config: actions, rewards, dones, drone dict order,
                                positions, charge, packet, ground, MT index, obs

Usage:  python oracle/gen_golden.py      (takes ~1 minute)
"""
from __future__ import annotations

import math
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "gymshim"))
sys.path.insert(0, "/root/reference")

from torch_impl.env.env import DeliveryDrones  # noqa: E402
from torch_impl.env.wrappers import WindowedGridView  # noqa: E402
from torch_impl.helpers.rl_helpers import set_seed  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

OBJ = {"skyscrapers": 2, "stations": 3, "dropzones": 4, "packets": 5}


def full_params(**kw):
    p = {
        'drone_density': 0.05, 'n_drones': 3, 'pickup_reward': 0, 'delivery_reward': 1,
        'crash_reward': -1, 'charge_reward': -0.1, 'discharge': 10, 'charge': 20,
        'packets_factor': 3, 'dropzones_factor': 2, 'stations_factor': 2,
        'skyscrapers_factor': 3, 'rgb_render_rescale': 1.0,
    }
    p.update(kw)
    return p


def snapshot(env):
    """Decode the reference env's dicts into arrays (drone vectors by index,
    dict order as a list of indices, ground codes)."""
    e = env.env if hasattr(env, "env") and not isinstance(env, DeliveryDrones) else env
    G, N = e.side_size, e.n_drones
    ground = np.zeros((G, G), dtype=np.uint8)
    for name, code in OBJ.items():
        for (y, x) in getattr(e, name):
            assert ground[y, x] == 0
            ground[y, x] = code
    order = np.zeros(N, dtype=np.int8)
    yy = np.zeros(N, dtype=np.uint8)
    xx = np.zeros(N, dtype=np.uint8)
    ch = np.zeros(N, dtype=np.int16)
    pk = np.zeros(N, dtype=bool)
    assert len(e.drones) == N
    for q, ((y, x), d) in enumerate(e.drones.items()):
        order[q] = d.index
        yy[d.index], xx[d.index], ch[d.index], pk[d.index] = y, x, d.charge, d.packet
    return ground, order, yy, xx, ch, pk


def mt_index():
    return random.getstate()[1][624]


def trajectory(params, seeds, steps, obs_every, action_seed):
    env = WindowedGridView(DeliveryDrones(params), radius=3)
    G, N = env.side_size, env.n_drones
    E = len(seeds)
    rng = np.random.default_rng(action_seed)
    actions = rng.integers(0, 5, size=(E, steps, N)).astype(np.int8)
    rec = {k: [] for k in ["ground", "order", "y", "x", "charge", "packet", "mtidx", "mt0", "rewards", "dones",
                           "obs", "obs_steps"]}
    obs_steps = [s for s in range(steps + 1) if s % obs_every == 0]
    for ei, s in enumerate(seeds):
        random.seed(int(s))
        mt0 = np.array(random.getstate()[1], dtype=np.uint32)
        obs = env.reset()
        snaps = [snapshot(env)]
        mtix = [mt_index()]
        rews, dns, obsl = [], [], []
        if 0 in obs_steps:
            obsl.append(np.stack([obs[i] for i in range(N)]).astype(np.float32))
        for t in range(steps):
            adict = {i: int(actions[ei, t, i]) for i in range(N)}
            obs, r, d, _, _ = env.step(adict)
            rews.append([float(r[i]) for i in range(N)])
            dns.append([bool(d[i]) for i in range(N)])
            snaps.append(snapshot(env))
            mtix.append(mt_index())
            if (t + 1) in obs_steps:
                obsl.append(np.stack([obs[i] for i in range(N)]).astype(np.float32))
        for k, idx in zip(["ground", "order", "y", "x", "charge", "packet"], range(6)):
            rec[k].append(np.stack([sn[idx] for sn in snaps]))
        rec["mtidx"].append(np.array(mtix, dtype=np.int16))
        rec["mt0"].append(mt0)
        rec["rewards"].append(np.array(rews, dtype=np.float64))
        rec["dones"].append(np.array(dns, dtype=bool))
        rec["obs"].append(np.stack(obsl))
    out = {k: np.stack(v) for k, v in rec.items() if k != "obs_steps"}
    out["obs_steps"] = np.array(obs_steps, dtype=np.int32)
    out["actions"] = actions
    out["seeds"] = np.array(seeds, dtype=np.int64)
    out["side"] = np.int32(G)
    pv = {k: v for k, v in params.items() if k != "rgb_render_rescale"}
    for k, v in pv.items():
        out["param_" + k] = np.float64(v)
    return out


def ref_tests():
    """The reference's own golden tests, replayed and captured as data."""
    out = {}
    # tests/torch_tests/test_windowedgridview.py:37-248
    p = full_params(n_drones=2, charge_reward=0.0)
    env = WindowedGridView(DeliveryDrones(p), radius=3)
    set_seed(env, 0)
    env.reset()
    acts = [{0: 3, 1: 4}, {0: 2, 1: 4}, {0: 2, 1: 4}]
    wins = []
    for a in acts:
        st, _, _, _, _ = env.step(a)
        wins.append(st[0].astype(np.float32))
    out["wgv_actions"] = np.array([[a[0], a[1]] for a in acts], dtype=np.int32)
    out["wgv_windows"] = np.stack(wins)

    # tests/torch_tests/test_env_single_drone.py:13-109
    p = full_params(n_drones=1, charge_reward=0.0)
    env = WindowedGridView(DeliveryDrones(p), radius=3)
    set_seed(env, 0)
    env.reset()
    seq = [3, 0, 0, 3, 3, 2, 3, 2, 2, 1, 1, 1, 1, 1] + [4] * 10
    ch, cp, rw = [], [], []
    for a in seq:
        _, r, _, _, _ = env.step({0: a})
        g, o, y, x, c, k = snapshot(env)
        ch.append(int(c[0])); cp.append(bool(k[0])); rw.append(float(r[0]))
    out["single_actions"] = np.array(seq, dtype=np.int32)
    out["single_charge"] = np.array(ch, dtype=np.int32)
    out["single_carry"] = np.array(cp, dtype=bool)
    out["single_reward"] = np.array(rw)

    # tests/torch_tests/test_env_multiple_drones.py:15-96 (drones 1..7 act by
    # RandomAgent -> env.action_space.sample(): gym PCG64 seeded by set_seed)
    p = full_params(n_drones=8)
    env = WindowedGridView(DeliveryDrones(p), radius=3)
    set_seed(env, 0)
    env.reset()
    scripted = [4, 1, 2, 3, 3, 2, 3, 3, 3, 3]
    acts, ch, cp, rw, dn = [], [], [], [], []
    for t in range(len(scripted)):
        a = {i: env.action_space.sample() for i in range(8)}
        a[0] = scripted[t]
        acts.append([a[i] for i in range(8)])
        _, r, d, _, _ = env.step(a)
        g, o, y, x, c, k = snapshot(env)
        ch.append(c.astype(np.int32)); cp.append(k.copy()); rw.append([float(r[i]) for i in range(8)])
        dn.append([bool(d[i]) for i in range(8)])
    out["multi_actions"] = np.array(acts, dtype=np.int32)
    out["multi_charge"] = np.stack(ch)
    out["multi_carry"] = np.stack(cp)
    out["multi_reward"] = np.array(rw)
    out["multi_done"] = np.array(dn)
    return out


CONFIGS = {
    # name: (params, seeds, steps, obs_every)
    "c1_g8_n4": (full_params(n_drones=4, drone_density=4 / 64), [0], 1000, 50),
    "c2_g16_n8": (full_params(n_drones=8, drone_density=8 / 256), list(range(8)), 200, 25),
    "c4_g32_n16": (full_params(n_drones=16, drone_density=16 / 1024), [0, 1, 2, 3], 100, 50),
    "c5_g64_n32": (full_params(n_drones=32, drone_density=32 / 4096), [0, 1], 60, 30),
    "t_g5_n1": (full_params(n_drones=1), [0, 1, 2], 200, 50),
    "t_g7_n2": (full_params(n_drones=2), [0, 1, 2], 200, 50),
    "t_g11_n6": (full_params(n_drones=6), [845, 99, 65], 300, 50),
    "t_g13_n8": (full_params(n_drones=8), [0, 5], 200, 50),
    # dense / collision-heavy, non-default rewards & factors
    "t_dense_n8": (full_params(n_drones=8, drone_density=0.08, pickup_reward=0.5, charge_reward=-0.25,
                               discharge=15, charge=30), [3, 4, 5], 300, 50),
    # Random.sample pool branch (n <= setsize): 2 drones on 5x5, 6 skyscrapers
    "t_pool_n2": (full_params(n_drones=2, drone_density=0.08, packets_factor=2, dropzones_factor=1,
                              stations_factor=1), [0, 1, 2, 3], 100, 50),
    "t_factors_n5": (full_params(n_drones=5, drone_density=0.1, packets_factor=1, dropzones_factor=1,
                                 stations_factor=3, skyscrapers_factor=1, discharge=25), [7, 8], 200, 50),
    "t_n33": (full_params(n_drones=33, drone_density=0.05), [11], 100, 50),
}


def main():
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "ref_tests.npz"), **ref_tests())
    for name, (p, seeds, steps, oe) in CONFIGS.items():
        d = trajectory(p, seeds, steps, oe, action_seed=1234 + len(name))
        path = os.path.join(OUT, f"traj_{name}.npz")
        np.savez_compressed(path, **d)
        print(f"{name}: G={int(d['side'])} N={p['n_drones']} envs={len(seeds)} steps={steps} "
              f"-> {os.path.getsize(path) / 1024:.0f} KiB; pool_branch="
              f"{(int(d['side'])**2 - p['skyscrapers_factor'] * p['n_drones']) <= _setsize(p['n_drones'])}")


def _setsize(k):
    s = 21
    if k > 5:
        s += 4 ** math.ceil(math.log(k * 3, 4))
    return s


if __name__ == "__main__":
    main()
