"""Helpers for the committed golden fixtures (tests/golden/, made by
oracle/gen_golden.py from the reference itself)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

PARAM_KEYS = ["drone_density", "n_drones", "pickup_reward", "delivery_reward", "crash_reward", "charge_reward",
              "discharge", "charge", "packets_factor", "dropzones_factor", "stations_factor", "skyscrapers_factor"]


def traj_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, "traj_*.npz")))


def load_traj(name):
    with np.load(os.path.join(GOLDEN, f"traj_{name}.npz")) as z:
        return {k: z[k] for k in z.files}


def load_ref_tests():
    with np.load(os.path.join(GOLDEN, "ref_tests.npz")) as z:
        return {k: z[k] for k in z.files}


def traj_params(d):
    """Reference env_params dict (torch_impl DEFAULT_CONFIG keys) of a fixture."""
    p = {k: d["param_" + k].item() for k in PARAM_KEYS}
    for k in ["n_drones", "discharge", "charge", "packets_factor", "dropzones_factor", "stations_factor",
              "skyscrapers_factor"]:
        p[k] = int(p[k])
    return p


def oracle_params(d):
    from oracle.oracle import Params
    p = traj_params(d)
    return Params(side=int(d["side"]), n_drones=p["n_drones"], charge=p["charge"], discharge=p["discharge"],
                  packets_factor=p["packets_factor"], dropzones_factor=p["dropzones_factor"],
                  stations_factor=p["stations_factor"], skyscrapers_factor=p["skyscrapers_factor"],
                  pickup_reward=p["pickup_reward"], delivery_reward=p["delivery_reward"],
                  crash_reward=p["crash_reward"], charge_reward=p["charge_reward"])


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name)) as z:
        return {k: z[k] for k in z.files}


def reset_configs():
    """Configs of reset_states.npz (oracle/gen_reset_mt_golden.py): name -> (side, n_drones)."""
    d = load_npz("reset_states.npz")
    return {k[:-6]: (int(d[k]), int(d[k[:-6] + "__n"])) for k in d if k.endswith("__side")}


def mt_sha(words625):
    """sha256 of the 624 MT state words (little-endian u32), as the fixture stores it."""
    import hashlib
    return np.frombuffer(hashlib.sha256(np.asarray(words625[:624], dtype="<u4").tobytes()).digest(), np.uint8)
