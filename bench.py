#!/usr/bin/env python3
"""Benchmark: batched DroneRL env step (+ fused windowed observation) on MI355X.

Metric (BASELINE.json): env-steps/s (= obs/s, train_jax.py:234) at
num_envs = 65536 per GPU (config C3: 16x16 grid, 8 drones), 1/2/4/8 GPUs.

One "step" = one drl_step launch over every env of the rank: moves,
collisions, pickup/delivery, battery, rewards, dones, respawns (the CPython
MT19937 streams included) and the fused observation of drone 0 (K=1, the
window train_jax.py:55-56 feeds the DQN).  Actions are synthetic uniform
{0..4}, generated before the timed region and resident in HBM.

Launch:  python bench.py [--gpus 1] [--steps 500] [--warmup 50]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); ~6300 achievable
CONFIGS = {
    # name: (grid, drones, envs per GPU, obs_k)
    "c2": (16, 8, 4096, 1),
    "c3": (16, 8, 65536, 1),
    "c4": (32, 16, 65536, 1),      # 262144 over 4 GPUs
    "c5": (64, 32, 131072, 1),     # 2**20 over 8 GPUs
}


def algorithmic_bytes(G: int, N: int, K: int, W: int = 7):
    """read R = G^2 + 4N + N per env-step; writes
    W = G^2 + 4N + 4N + N + obs (K * W*W*6 f32)."""
    R = G * G + 4 * N + N
    Wb = G * G + 4 * N + 4 * N + N + K * W * W * 6 * 4
    return R, Wb


# DRL_DIST_BACKEND=gloo rehearses the multi-rank path where there are fewer
# GPUs than ranks (ranks share devices round-robin; the max-over-ranks
# reductions then run on host tensors).  The driver's runs use nccl (RCCL).
DIST_BACKEND = os.environ.get("DRL_DIST_BACKEND", "nccl")


def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if DIST_BACKEND == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group(DIST_BACKEND)
    else:
        torch.cuda.set_device(local)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device="cuda" if DIST_BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(v: float, world: int) -> float:
    return -max_over_ranks(-v, world)


def under_profiler():
    """True inside a rocprofv3 run: its preloaded tool has initialised the GPU
    in this process, so a nested rocprofv3 child (which execs its target) must
    not start; the committed profile is reported instead."""
    pre = os.environ.get("LD_PRELOAD", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def measure_traffic(args):
    """HBM bytes per drl_step launch from rocprofv3 PMC passes of this same
    bench command (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in
    separate passes, FETCH_SIZE doubled for gfx950, KiB -> bytes).  Runs as
    child processes before this process touches the GPU; returns None when
    rocprofv3 is absent or a pass fails (the caller then reports the committed
    profile, labelled as such)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3")
                                         else None)
    if prof is None or under_profiler():
        return None
    child = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", "20", "--warmup", "3",
             "--no-cpu-baseline", "--no-reset-bench", "--no-dqn", "--rollout-chunk", "0", "--loop-segments", "0",
             "--no-pmc-traffic", "--cached-steps", "0"]
    if args.envs:
        child += ["--envs", str(args.envs)]
    child.append("--obs-stream" if args.obs_stream else "--obs-cached")
    if args.obs_k >= 0:
        child += ["--obs-k", str(args.obs_k)]
    vals = {}
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    with tempfile.TemporaryDirectory(prefix="drl_pmc_") as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "drl_step_kernel", "-d", d, "-o", "run",
                   "--output-format", "csv", "--"] + child
            try:
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=150, env=env,
                                   cwd=REPO)
            except subprocess.TimeoutExpired:
                print(f"pmc pass {ctr}: timed out", file=sys.stderr)
                return None
            if r.returncode != 0:
                print(f"pmc pass {ctr}: rc={r.returncode} {r.stderr.decode(errors='replace')[-300:]}",
                      file=sys.stderr)
                return None
            xs = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    if "drl_step_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        xs.append(float(row["Counter_Value"]))
            if not xs:
                return None
            vals[ctr] = sum(xs) / len(xs)
    read_b = 2 * vals["FETCH_SIZE"] * 1024
    write_b = vals["WRITE_SIZE"] * 1024
    return {"bytes_per_launch": read_b + write_b, "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
            "fetch_size_kib": vals["FETCH_SIZE"], "write_size_kib": vals["WRITE_SIZE"],
            "source": "measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate child runs "
                      "of this bench, 20 steps), traffic = 2*FETCH_SIZE + WRITE_SIZE"}


def load_traffic(cfg_name: str):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/),
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, or None."""
    path = os.path.join(REPO, "profiles", f"pmc_{cfg_name}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """CPUs this process can actually use: the scheduler affinity, capped by
    a cgroup CPU quota when one is set (a GPU lease's CPU share: the affinity
    mask there lists the whole machine, and threads beyond the quota only
    time-slice)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, period = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(period)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, -(-q // period))
        except (OSError, ValueError):
            pass
    n = min(aff, quota) if quota else aff
    return n, f"affinity {aff} CPUs" + (f", cgroup CPU quota {quota}" if quota else ", no cgroup CPU quota")


def cpu_baseline(G, N, K, seconds: float):
    """The oracle (C restatement of torch_impl step + WindowedGridView) on host
    cores, bounded sample; 'port' baseline (the same workload
    with a static env partition over the host threads, plus a 1-thread figure)."""
    from oracle.oracle import Params, rollout
    threads, cpu_note = host_cpus()  # every host core this process may use
    p = Params(side=G, n_drones=N)
    E = max(4096, 128 * threads)

    def timed(envs, steps, nthreads):
        t0 = time.perf_counter()
        rollout(p, envs, steps, nthreads=nthreads, want_state=False, obs_k=K, action_seed=1)
        return time.perf_counter() - t0

    # per-step cost from two probe lengths (the reset and thread start-up cancel)
    t_a, t_b = timed(E, 20, threads), timed(E, 220, threads)
    per_step = max((t_b - t_a) / 200, 1e-6)
    steps = max(10, int((seconds - max(t_a - 20 * per_step, 0.0)) / per_step))
    dt = timed(E, steps, threads)
    if dt < 0.6 * seconds:  # early-episode steps cost more than steady state: one corrective run
        steps = int(steps * seconds / dt)
        dt = timed(E, steps, threads)
    # single thread, a quarter of the envs, ~1/4 of the time budget
    e1 = E // 4
    t1a, t1b = timed(e1, 4, 1), timed(e1, 24, 1)
    s1 = max(2, int(seconds / 4 / max((t1b - t1a) / 20, 1e-6)))
    d1 = timed(e1, s1, 1)
    if d1 < 0.15 * seconds:
        s1 = int(s1 * seconds / 4 / d1)
        d1 = timed(e1, s1, 1)
    return {"value": E * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{E} envs x {steps} steps of reset + step()+obs(K={K}) at {G}x{G}/{N} drones, "
                      f"{threads} host threads (static env partition), {dt:.1f}s wall",
            "cores_basis": cpu_note,
            "single_thread_value": e1 * s1 / d1,
            "single_thread_sample": f"{e1} envs x {s1} steps, 1 thread, {d1:.1f}s wall",
            "cpu_model": cpu_model()}


def dqn_consumer_bench(env, actions, rewards, dones, obs, warmup, steps, stream):
    """the C3 loop's consumer of the observation, timed
    separately from the env step.  (1) drl_qnet_act alone on the resident obs
    (dense 294->128->64->5 on MFMA, epsilon-greedy, writes actions[:, 0]):
    HBM-bound on reading the obs (E * W*W*6 f32); (2) the train_jax.py:42-64
    loop shape per step: act -> step + obs -> replay add_many (capacity 10000)."""
    from dronerl_amd.dqn import QNetwork, ReplayBuffer
    E = env.num_envs
    D = obs[0].numel()
    net = QNetwork(D, (128, 64), device=env.device, generator=torch.Generator().manual_seed(0))
    rb = ReplayBuffer(10000, D, env.device)
    flat = obs.reshape(E, -1)
    a0 = actions[0]
    for t in range(warmup):
        net.act(flat, 0.1, seed=1, step=t, actions=a0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    for t in range(steps):
        net.act(flat, 0.1, seed=1, step=t, actions=a0)
    ev[1].record(stream)
    # loop shape: act on obs_t, step writing obs_t+1 into the other buffer, add the transition
    bufs = [obs, torch.empty_like(obs)]
    ev[2].record(stream)
    for t in range(steps):
        cur, nxt = bufs[t & 1], bufs[(t + 1) & 1]
        a = actions[t % actions.shape[0]]
        net.act(cur.reshape(E, -1), 0.1, seed=1, step=t, actions=a)
        env.step(a, obs_k=1, rewards=rewards, dones=dones, obs=nxt)
        rb.add_many(cur, a, rewards, nxt, dones)
    ev[3].record(stream)
    torch.cuda.synchronize()
    env.check_errors()
    # the same act with the reference's f32 numerics (DRL_QNET_F32)
    net32 = QNetwork(D, (128, 64), device=env.device, generator=torch.Generator().manual_seed(0), precision="f32")
    for t in range(warmup):
        net32.act(flat, 0.1, seed=1, step=t, actions=a0)
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record(stream)
    for t in range(steps):
        net32.act(flat, 0.1, seed=1, step=t, actions=a0)
    f1.record(stream)
    torch.cuda.synchronize()
    act32_s = f0.elapsed_time(f1) / 1e3 / steps
    act_s = ev[0].elapsed_time(ev[1]) / 1e3 / steps
    loop_s = ev[2].elapsed_time(ev[3]) / 1e3 / steps
    read = E * D * 4
    return {"net": f"dense {D}->128->64->5, bf16 MFMA (f32 accumulate)", "act_us": act_s * 1e6,
            "act_roofline": {"bound": "hbm", "achieved": read / act_s / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": read / act_s / 1e9 / PEAK_HBM_GBS,
                             "algorithmic_bytes_per_env": D * 4 + 4},
            "act_f32_us": act32_s * 1e6,
            "act_f32_roofline": {"bound": "hbm", "achieved": read / act32_s / 1e9, "peak": PEAK_HBM_GBS,
                                 "unit": "GB/s", "frac": read / act32_s / 1e9 / PEAK_HBM_GBS},
            "act_f32_note": "precision='f32' (DRL_QNET_F32): fp16 hi/lo split operands, 3 MFMAs per product tile, "
                            "Q to f32 rounding (the reference's f32 nets)",
            "loop_us_per_step": loop_s * 1e6, "loop_env_steps_per_s": E / loop_s,
            "loop": "act(obs_t) -> step + obs(K=1) -> replay add_many(obs_t, a, r, obs_t+1, done), capacity 10000"}


def rollout_bench(env, actions, K, warmup_steps, steps, chunk: int, R: int, Wb: int, world: int):
    """drl_rollout (jax run_steps shape, env.py:252-272, plus every step's
    rewards, dones and obs(K)): `chunk` steps per launch with the state on chip
    between them, the same pre-generated actions as the per-step loop, every
    step's outputs stored ([chunk, E, ...] buffers).  Timed like the main loop
    (barrier + synchronize, max over ranks)."""
    E, N, dev = env.num_envs, env.n_drones, env.device
    W = env.layout.obs_window
    rew = torch.empty((chunk, E, N), dtype=torch.float32, device=dev)
    don = torch.empty((chunk, E, N), dtype=torch.uint8, device=dev)
    obs = torch.empty((chunk, E, max(K, 1), W, W, 6), dtype=torch.float32, device=dev) if K else None
    T = actions.shape[0]

    def run(t0, n):
        a = actions[t0 % T: t0 % T + n] if t0 % T + n <= T else actions[:n]
        env.rollout(a, obs_k=K, rewards=rew[:n], dones=don[:n], obs=obs[:n] if K else None)

    for t0 in range(0, warmup_steps, chunk):
        run(t0, min(chunk, warmup_steps - t0))
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_wall = time.perf_counter()
    e0.record(stream)
    done = 0
    while done < steps:
        n = min(chunk, steps - done)
        run(warmup_steps + done, n)
        done += n
    e1.record(stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    wall = max_over_ranks(time.perf_counter() - t_wall, world)
    env.check_errors()
    ev_s = e0.elapsed_time(e1) / 1e3
    per_step = ev_s / steps
    return {"value": E * world * steps / wall, "unit": "env-steps/s", "steps": steps, "steps_per_launch": chunk,
            "ms_per_step": wall / steps * 1e3,
            "kernel": "drl_rollout_kernel", "avg_launch_us": ev_s / -(-steps // chunk) * 1e6,
            "roofline": {"bound": "hbm", "achieved": E * R / per_step / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": E * R / per_step / 1e9 / PEAK_HBM_GBS,
                         "achieved_read_plus_write": E * (R + Wb) / per_step / 1e9,
                         "frac_read_plus_write": E * (R + Wb) / per_step / 1e9 / PEAK_HBM_GBS,
                         "note": "same per-env-step algorithmic bytes as drl_step (SURVEY.md §8 D3); the state is "
                                 "read and written once per launch, so HBM traffic per step is lower"}}


# diagnostic: the train loop's step with streaming observation stores (A/B of
# env.step()'s store mode where the act kernel reads the observation next)
LOOP_OBS_STREAM = {"0": False, "1": True}.get(os.environ.get("DRL_LOOP_OBS_STREAM", ""))


class TrainSegment:
    """One segment of the train_jax.py:38-113 loop minus the learner (SURVEY.md
    §8 D2; C5: "multi-step loop, hipGraph of step+obs+act"): per step,
    synthetic actions for every drone, the epsilon-greedy DQN action for drone
    0 (dense 294->128->64->5), step + obs(K=1), replay add_many of the drone-0
    transition; after `seg` steps a reset of every env (reset_env_every,
    train_jax.py:101-113) and its first observation.

    fused=True (one stream only): the synthetic actions of drones 1..N-1 are
    written by the act launch itself (drl_qnet_act_synth), one kernel fewer
    per step with the same action rows.

    parallel=True: the synthetic actions and the replay add run on two side
    streams, joined to the act -> step chain by events.  Observations, actions,
    rewards and dones rotate through 3 buffers, so step t only waits for the
    replay add of step t-2 and the actions of step t are drawn while step t-1
    runs.  parallel=False issues the same calls in the same order on one
    stream with 2 buffers; both leave identical state and replay contents
    (tests/test_gpu_parity.py::test_train_segment_parallel_matches_serial)."""

    def __init__(self, env, seg: int, parallel: bool = False, net=None, rb=None, fused: bool = True):
        from dronerl_amd.dqn import QNetwork, ReplayBuffer
        E, N, dev = env.num_envs, env.n_drones, env.device
        W = env.layout.obs_window
        D = W * W * 6
        self.env, self.seg, self.parallel, self.E = env, seg, parallel, E
        self.fused = fused and not parallel
        # parallel branches need 3 rotating buffers (see above); on one stream 2
        # suffice, and the third 77 MB observation buffer costs MALL hits (C3
        # loop 79.4 vs 74.4 us per step)
        self.NB = 3 if parallel else 2
        self.net = net or QNetwork(D, (128, 64), device=dev, generator=torch.Generator().manual_seed(0))
        self.rb = rb or ReplayBuffer(10000, D, dev)
        self.acts = [torch.empty((E, N), dtype=torch.int32, device=dev) for _ in range(self.NB)]
        self.rewards = [torch.empty((E, N), dtype=torch.float32, device=dev) for _ in range(self.NB)]
        self.dones = [torch.empty((E, N), dtype=torch.uint8, device=dev) for _ in range(self.NB)]
        self.obs = [torch.empty((E, 1, W, W, 6), dtype=torch.float32, device=dev) for _ in range(self.NB)]
        env.get_obs(1, out=self.obs[0])
        self.s_syn, self.s_rep = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def _synth(self, t):
        self.env.synth_actions(seed=2024, step=t, out=self.acts[t % self.NB])

    def _act_step(self, t):
        b, nb = t % self.NB, (t + 1) % self.NB
        self.net.act(self.obs[b].reshape(self.E, -1), 0.1, seed=7, step=t, env_offset=self.env.env_offset,
                     actions=self.acts[b], synth=(2024, t) if self.fused else None)
        self.env.step(self.acts[b], obs_k=1, rewards=self.rewards[b], dones=self.dones[b], obs=self.obs[nb],
                      obs_stream=LOOP_OBS_STREAM)  # None: env.step()'s default

    def _replay(self, t):
        b, nb = t % self.NB, (t + 1) % self.NB
        self.rb.add_many(self.obs[b], self.acts[b], self.rewards[b], self.obs[nb], self.dones[b])

    def run(self):
        main = torch.cuda.current_stream(self.env.device)
        if not self.parallel:
            for t in range(self.seg):
                if not self.fused:
                    self._synth(t)
                self._act_step(t)
                self._replay(t)
        else:
            ev_syn = [torch.cuda.Event() for _ in range(self.seg)]
            ev_step = [torch.cuda.Event() for _ in range(self.seg)]
            ev_rep = [torch.cuda.Event() for _ in range(self.seg)]
            self.s_syn.wait_stream(main)
            self.s_rep.wait_stream(main)
            for t in range(self.seg):
                with torch.cuda.stream(self.s_syn):
                    if t >= self.NB:  # acts[t % 3] was last read by the replay add of step t-3
                        self.s_syn.wait_event(ev_rep[t - self.NB])
                    self._synth(t)
                    ev_syn[t].record(self.s_syn)
                main.wait_event(ev_syn[t])
                if t >= 2:  # step t overwrites obs[(t+1) % 3], read by the replay add of step t-2
                    main.wait_event(ev_rep[t - 2])
                self._act_step(t)
                ev_step[t].record(main)
                with torch.cuda.stream(self.s_rep):
                    self.s_rep.wait_event(ev_step[t])
                    self._replay(t)
                    ev_rep[t].record(self.s_rep)
            main.wait_stream(self.s_syn)
            main.wait_stream(self.s_rep)
        self.env.reset(seed=None)
        self.env.get_obs(1, out=self.obs[0])


def train_loop_bench(env, reps: int, seg: int = 100, parallel: bool = False, fused: bool = True):
    """TrainSegment captured once as a HIP graph (no host work per step) and
    replayed.  Counters (action stream step, epsilon draws, replay cursor) are
    baked into the capture, so replays repeat them: the work per step is the
    same, the action stream repeats every segment."""
    dev = env.device
    loop = TrainSegment(env, seg, parallel=parallel, fused=fused)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        loop.run()  # eager warm-up on the capture stream
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loop.run()
    g.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize(dev)
    env.check_errors()
    dt = e0.elapsed_time(e1) / 1e3
    E = env.num_envs
    branches = ("synthetic actions and replay add_many on parallel graph branches, 3 rotating buffers"
                if parallel else "one stream" + ("; synthetic actions inside the act launch" if fused else ""))
    return {"env_steps_per_s": E * seg * reps / dt, "us_per_step": dt / (seg * reps) * 1e6,
            "segments": reps, "steps_per_segment": seg,
            "loop": f"hipGraph of {seg} x [synth actions -> qnet act (drone 0) -> step + obs(K=1) -> "
                    f"replay add_many] + reset + obs, replayed {reps}x ({branches}; learner not included)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=0, help="override envs per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-reset-bench", action="store_true")
    ap.add_argument("--no-dqn", action="store_true", help="skip the DQN-consumer measurement (SURVEY.md §8 F1)")
    ap.add_argument("--rollout-chunk", type=int, default=100,
                    help="steps per drl_rollout launch for the rollout measurement (0 = skip)")
    ap.add_argument("--loop-segments", type=int, default=3,
                    help="train-loop graph replays (100 steps + reset each; 0 = skip)")
    ap.add_argument("--unfused-act", action="store_true",
                    help="train loop: synthetic actions as their own launch instead of inside the act launch")
    ap.add_argument("--parallel-loop", action="store_true",
                    help="train loop with synth / replay on parallel graph branches (measured slower: the step "
                         "kernel fills every CU in one generation, and co-running kernels delay its waves)")
    ap.add_argument("--obs-stream", action="store_true",
                    help="write the per-step observation with streaming stores (DRL_STEP_OBS_STREAM); default: "
                         "env.step()'s mode (cached at 8 lanes per env, streaming at >= 16)")
    ap.add_argument("--obs-cached", action="store_true", help="write the per-step observation with cached stores")
    ap.add_argument("--obs-k", type=int, default=-1,
                    help="diagnostic: observed drones per step (default: the config's; 0 = step without obs)")
    ap.add_argument("--cached-steps", type=int, default=200,
                    help="also time this many steps with the other observation store mode and report them under "
                         "`streaming_obs` (or `cached_obs` with --obs-stream) (0 = skip)")
    ap.add_argument("--no-pmc-traffic", action="store_true",
                    help="do not run the rocprofv3 FETCH_SIZE / WRITE_SIZE passes for roofline.traffic")
    args = ap.parse_args()

    traffic_run = None
    if (not args.no_pmc_traffic and int(os.environ.get("WORLD_SIZE", "1")) == 1
            and os.environ.get("DRL_BENCH_PMC", "1") != "0"):
        traffic_run = measure_traffic(args)  # child processes, before this one touches the GPU

    rank, world, local = dist_init()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    from dronerl_amd._native import DRL_STEP_OBS_STREAM, lib

    G, N, E, K = CONFIGS[args.config]
    if args.envs:
        E = args.envs
    if args.obs_k >= 0:
        K = args.obs_k
    p = EnvParams(n_drones=N, grid_size=G)
    dev = torch.device("cuda", local)
    env = BatchedDeliveryDrones(p, E, device=dev, env_offset=rank * E)
    env.reset(seed=0)
    T = args.warmup + args.steps
    # synthetic actions for every step, resident in HBM before timing
    actions = torch.empty((T, E, N), dtype=torch.int32, device=dev)
    for t in range(T):
        env.synth_actions(seed=2024, step=t, out=actions[t])
    if not args.obs_stream and not args.obs_cached:  # env.step()'s default store mode
        args.obs_stream = env.default_obs_stream
    W = env.layout.obs_window
    rewards = torch.empty((E, N), dtype=torch.float32, device=dev)
    dones = torch.empty((E, N), dtype=torch.uint8, device=dev)
    obs = torch.empty((E, max(K, 1), W, W, 6), dtype=torch.float32, device=dev)

    # fast path: ctypes arguments built once; only the actions pointer moves
    L = lib()
    cp = ctypes.byref(env._cp)
    st = env.state.c()
    sp = ctypes.byref(st)
    a_ptrs = [ctypes.c_void_p(actions[t].data_ptr()) for t in range(T)]
    r_p, d_p, o_p = (ctypes.c_void_p(x.data_ptr()) for x in (rewards, dones, obs))
    if K == 0:
        o_p = None
    e_p = ctypes.c_void_p(env.err.data_ptr())
    stream = torch.cuda.current_stream(dev)
    s_p = ctypes.c_void_p(stream.cuda_stream)

    # cached observation stores (env.step()'s default, what a train_jax-style
    # caller gets) unless --obs-stream; the other mode is timed after it
    flags = DRL_STEP_OBS_STREAM if args.obs_stream else 0

    # the respawn-candidate rings are topped up every refill_every steps (what
    # env.step() does), as a separate drl_refill launch bracketed by its own
    # events, so the step kernel's average duration can be separated from it
    refill_every = env.refill_every
    refill_ev = []  # (start, end) event pairs of the timed region's refills

    def run(t, timed=False):
        rc = L.drl_step_ex(cp, sp, a_ptrs[t], r_p, d_p, o_p, K, e_p, flags, s_p)
        if rc:
            raise RuntimeError(L.drl_last_error().decode())
        if refill_every > 0 and (t + 1) % refill_every == 0:
            if timed:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(stream)
            rc = L.drl_refill(cp, sp, s_p)
            if rc:
                raise RuntimeError(L.drl_last_error().decode())
            if timed:
                ev[1].record(stream)
                refill_ev.append(ev)

    for t in range(args.warmup):
        run(t)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for t in range(args.warmup, T):
        run(t, timed=True)
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    env.check_errors()
    wall_max = max_over_ranks(wall, world)

    total_env_steps = E * world * args.steps
    value = total_env_steps / wall_max
    refill_ms = sum(a.elapsed_time(b) for a, b in refill_ev)
    launch_s = (ev_ms - refill_ms) / 1e3 / args.steps  # average drl_step duration on this stream
    refill = {"every": refill_every, "launches": len(refill_ev),
              "avg_launch_us": refill_ms / max(len(refill_ev), 1) * 1e3,
              "per_step_us": refill_ms / args.steps * 1e3,
              "note": "drl_refill (respawn-candidate rings) launches inside the timed region: in value and "
                      "ms_per_step, not in roofline.avg_launch_us (the drl_step kernel alone)"}
    R, Wb = algorithmic_bytes(G, N, K, W)
    achieved = E * R / launch_s / 1e9
    achieved_rw = E * (R + Wb) / launch_s / 1e9

    # the other observation store mode, same steps
    cached = None
    if args.cached_steps > 0 and K > 0:
        flags_main = flags
        flags = 0 if args.obs_stream else DRL_STEP_OBS_STREAM
        nc = min(args.cached_steps, args.steps)
        for t in range(min(args.warmup, 20)):
            run(t)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tc = time.perf_counter()
        c0.record(stream)
        for t in range(args.warmup, args.warmup + nc):
            run(t)
        c1.record(stream)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        cwall = max_over_ranks(time.perf_counter() - tc, world)
        env.check_errors()
        flags = flags_main
        c_launch = c0.elapsed_time(c1) / 1e3 / nc  # (refill share included)
        cached = {"value": E * world * nc / cwall, "unit": "env-steps/s", "steps": nc,
                  "ms_per_step": cwall / nc * 1e3, "avg_launch_us": c_launch * 1e6,
                  "frac": E * algorithmic_bytes(G, N, K, W)[0] / c_launch / 1e9 / PEAK_HBM_GBS,
                  "obs_stores": "cached" if args.obs_stream else "streaming",
                  "note": "the other observation store mode, same steps and results; `value` uses env.step()'s "
                          "default (cached stores at 8 lanes per env, streaming at >= 16: the faster one in "
                          "the train loop, profiles/r02_store_mode/)"}

    # resets (train_jax.py:101-113 resets every 100 steps in C5): timed separately
    resets_per_s = None
    if not args.no_reset_bench:
        env.reset(seed=None)
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record(stream)
        nres = 3
        for _ in range(nres):
            env.reset(seed=None)
        r1.record(stream)
        torch.cuda.synchronize()
        resets_per_s = E * world * nres / (r0.elapsed_time(r1) / 1e3)

    dqn = None
    if K >= 1 and not args.no_dqn:
        dqn = dqn_consumer_bench(env, actions, rewards, dones, obs, args.warmup, min(args.steps, 200), stream)

    roll = None
    if args.rollout_chunk > 0:
        env.reset(seed=0)
        roll = rollout_bench(env, actions, K, args.warmup, args.steps, args.rollout_chunk, R, Wb, world)
        if K > 0:  # jax run_steps exactly (no observation): rewards/dones of every step only
            env.reset(seed=0)
            R0, W0 = algorithmic_bytes(G, N, 0, W)
            r0 = rollout_bench(env, actions, 0, args.warmup, args.steps, args.rollout_chunk, R0, W0, world)
            roll["no_obs"] = {k: r0[k] for k in ("value", "ms_per_step")}

    loop = None
    if args.loop_segments > 0 and not args.no_dqn and K >= 1:
        loop = train_loop_bench(env, args.loop_segments, parallel=args.parallel_loop, fused=not args.unfused_act)
        loop["env_steps_per_s"] = min_over_ranks(loop["env_steps_per_s"], world) * world
        loop["n_gpus"] = world

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(G, N, K, args.cpu_seconds)

    traffic_src = None
    if traffic_run is not None:
        traffic, traffic_src = traffic_run["bytes_per_launch"], traffic_run
    else:
        traffic = load_traffic(args.config)
        if traffic is not None:
            traffic_src = {"source": f"committed profiles/pmc_{args.config}.json (an earlier run; no rocprofv3 pass "
                                     "in this one)"}
    if rank == 0:
        with open(os.path.join(REPO, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
        out = {
            "metric": metric,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic uniform random actions (counter hash), envs seeded random.seed(env index)",
            "config": {"workload": f"{args.config.upper()}: {G}x{G} grid, {N} drones, {E} envs/GPU, "
                                   f"step + fused obs(K={K})",
                       "grid": G, "n_drones": N, "num_envs_per_gpu": E, "num_envs_total": E * world,
                       "obs_k": K, "obs_stores": "streaming" if args.obs_stream else "cached",
                       "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS,
                         "traffic": traffic,
                         "kernel": "drl_step_kernel", "avg_launch_us": launch_s * 1e6,
                         "algorithmic_read_bytes_per_env_step": R,
                         "algorithmic_write_bytes_per_env_step": Wb,
                         "achieved_read_plus_write": achieved_rw,
                         "frac_read_plus_write": achieved_rw / PEAK_HBM_GBS,
                         "frac_ceiling": R / (R + Wb),
                         "note": "frac counts SURVEY.md §8 D3's read bytes R only: moving all R + W "
                                 "algorithmic bytes at the HBM peak would score frac_ceiling = R / (R + W). W counts "
                                 "a full ground write-back but the kernel writes only the changed cells, so the "
                                 "read+write figure can exceed the peak at large grids (C5). Measured HBM bytes "
                                 "per launch: traffic",
                         "traffic_detail": traffic_src},
            "refill": refill,
            ("cached_obs" if args.obs_stream else "streaming_obs"): cached,
            "cpu_baseline": cpu,
            "resets_per_s": resets_per_s,
            "dqn_consumer": dqn,
            "rollout": roll,
            "train_loop": loop,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
