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
         python bench.py --gpus N          (starts its own N ranks, below)
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints one JSON line on rank 0.

`--gpus N > 1` without a torch.distributed.run environment (no WORLD_SIZE):
this process becomes a launcher.  Before touching the GPU it runs
`torch.distributed.run --nproc-per-node N` as a child process (never an
exec), one rank per GPU over RCCL (train_jax.py:196-212: envs sharded over
the devices, num_envs % devices == 0, :399-402), relays rank 0's JSON line
and exits with the job's return code.
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


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_command(argv, n: int, port: int):
    """The child command of `bench.py --gpus N` (N > 1, no WORLD_SIZE): N ranks
    of this script under torch.distributed.run on one node, rendezvous on
    127.0.0.1, the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def needs_launch(args) -> bool:
    return args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child


def visible_gpus():
    """GPUs the ranks could use, counted without touching the HIP runtime (the
    launcher stays GPU-free): the KFD topology's GPU nodes (simd_count > 0),
    narrowed by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.
    None when the topology is unreadable (no check then)."""
    import glob
    n = 0
    nodes = glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")
    if not nodes:
        return None
    for f in nodes:
        try:
            for ln in open(f):
                k, _, v = ln.partition(" ")
                if k == "simd_count" and int(v) > 0:
                    n += 1
        except (OSError, ValueError):
            return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(argv, n: int) -> int:
    """Run the N-rank job as a child process (this process never initialises
    the GPU: argument parsing only), forward its output, print rank 0's JSON
    line (the only line starting with '{"metric"') last on stdout, and return
    the job's exit code: torch.distributed.run fails when any rank fails; a
    clean job without a JSON line is an error too."""
    import subprocess
    if DIST_BACKEND == "nccl":
        have = visible_gpus()
        if have is not None and have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible; nccl needs one GPU per rank "
                  "(DRL_DIST_BACKEND=gloo shares devices)", file=sys.stderr)
            return 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = launcher_command(argv, n, free_port())
    print("bench.py launcher: " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=REPO)
    lines = []
    for ln in p.stdout:
        if ln.startswith('{"metric"'):
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = p.wait()
    if rc == 0 and len(lines) != 1:
        print(f"bench.py launcher: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        rc = 1
    for ln in lines:
        print(ln, flush=True)
    return rc


def strong_split(total: int, world: int) -> int:
    """Envs per rank of the strong-scaling sub-record: `total` envs over the
    job, contiguous shards (train_jax.py:196-212), num_envs % devices == 0 as
    train_jax.py:401-402 requires."""
    if total <= 0 or world <= 0 or total % world:
        raise ValueError(f"the number of envs (={total}) needs to be divisible by the number of devices (={world})")
    return total // world


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


# torchrun's per-rank variables: a rocprofv3 child started by rank 0 must run
# as a plain single-process bench, not join the job's process group
TORCHRUN_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")

# (drl_refill_list_kernel: the refill's default form since round 3; drl_refill_kernel under DRL_REFILL_LIST=0)
PMC_KERNELS = ("drl_step_kernel", "drl_refill_list_kernel", "drl_refill_kernel")


def child_env():
    env = {k: v for k, v in os.environ.items() if k not in TORCHRUN_VARS and not k.startswith("TORCHELASTIC")}
    env["TMPDIR"] = os.environ.get("TMPDIR", "/tmp")
    local = os.environ.get("LOCAL_RANK")
    if local not in (None, "0"):  # the rank's own GPU (rank 0 is normally local rank 0)
        env["HIP_VISIBLE_DEVICES"] = local
    return env


def measure_traffic(args, names):
    """HBM bytes per launch of drl_step_kernel and drl_refill(_list)_kernel for each
    config in `names`, from rocprofv3 PMC passes of this same bench
    (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes,
    FETCH_SIZE doubled for gfx950, KiB -> bytes).  One child process per
    counter runs every config's step loop (`--pmc-child`, same store mode,
    same pre-roll and refill cadence as the timed loops) before this process
    touches the GPU; the child reports each config's launch grid sizes, which
    attribute the counter rows.  Returns None when rocprofv3 is absent or a
    pass fails (the caller then reports the committed profile, labelled)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3")
                                         else None)
    if prof is None or under_profiler():
        return None
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", ",".join(names), "--config", args.config,
             "--steps", "20", "--warmup", "3", "--envs", str(args.envs), "--c5-envs", str(args.c5_envs)]
    # the store mode: forced flags pass through; otherwise the child resolves
    # env.step()'s default itself, exactly as the timed loop does
    if args.obs_stream:
        child.append("--obs-stream")
    elif args.obs_cached:
        child.append("--obs-cached")
    if args.obs_k >= 0:
        child += ["--obs-k", str(args.obs_k)]
    rows = {}
    grids = None
    env = child_env()
    with tempfile.TemporaryDirectory(prefix="drl_pmc_") as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            cmd = [prof, "--pmc", ctr, "--kernel-include-regex", "|".join(PMC_KERNELS), "-d", d, "-o", "run",
                   "--output-format", "csv", "--"] + child
            try:
                r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=240, env=env,
                                   cwd=REPO)
            except subprocess.TimeoutExpired:
                print(f"pmc pass {ctr}: timed out", file=sys.stderr)
                return None
            if r.returncode != 0:
                print(f"pmc pass {ctr}: rc={r.returncode} {r.stderr.decode(errors='replace')[-300:]}",
                      file=sys.stderr)
                return None
            for ln in r.stdout.decode(errors="replace").splitlines():
                if ln.startswith("{\"pmc_child\""):
                    grids = json.loads(ln)["pmc_child"]
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    if row.get("Counter_Name") != ctr:
                        continue
                    kern = next((k for k in PMC_KERNELS if k in row.get("Kernel_Name", "")), None)
                    if kern:
                        rows.setdefault((ctr, kern, int(row["Grid_Size"])), []).append(float(row["Counter_Value"]))
    if not grids:
        return None
    out = {}
    for name, g in grids.items():
        rec = {}
        for kern, key in (("drl_step_kernel", "step_grid"), ("drl_refill_list_kernel", "refill_list_grid"),
                          ("drl_refill_kernel", "refill_grid")):
            f = rows.get(("FETCH_SIZE", kern, g[key]))
            w = rows.get(("WRITE_SIZE", kern, g[key]))
            if not f or not w:
                continue
            rd = 2 * sum(f) / len(f) * 1024
            wr = sum(w) / len(w) * 1024
            rec[kern] = {"bytes_per_launch": rd + wr, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                         "read_bytes_per_env": rd / g["envs"], "write_bytes_per_env": wr / g["envs"],
                         "launches": min(len(f), len(w))}
        if "drl_step_kernel" in rec:
            rec["envs"] = g["envs"]
            rec["source"] = ("measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate child "
                             "runs of this bench's step loop, 20 steps after a two-refill-cycle pre-roll), traffic = "
                             "2*FETCH_SIZE + WRITE_SIZE per launch")
            out[name] = rec
    return out or None


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
            "cpu_model": cpu_model(), "reference_torch_impl": reference_torch_impl(G, N)}


# the reference's own torch_impl step()+WindowedGridView, timed in the build container by
# oracle/time_reference_torch_impl.py (the reference cannot run on the GPU box): quoted, not measured here
REFERENCE_TIMING = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                "r06_reference_torch_impl.json")


def reference_torch_impl(G, N):
    try:
        with open(REFERENCE_TIMING) as f:
            ref = json.load(f)
    except (OSError, ValueError):
        return None
    for cfg in ref.get("configs", {}).values():
        if cfg.get("side") == G and cfg.get("n_drones") == N:
            return {"value": cfg["step_obs_env_steps_per_s"], "unit": "env-steps/s", "cores": ref.get("cores", 1),
                    "kind": "reference", "step_only_value": cfg["step_only_env_steps_per_s"],
                    "hardware": ref.get("hardware"), "different_hardware": True,
                    "sample": f"{cfg['timed_steps']} steps of one env, uniform random actions",
                    "source": "profiles/r06_reference_torch_impl.json (oracle/time_reference_torch_impl.py)"}
    return None


def dqn_consumer_bench(env, actions, rewards, dones, obs, warmup, steps, stream, precision="f32", input="obs"):
    """the C3 loop's consumer of the observation, timed
    separately from the env step.  (1) drl_qnet_act alone on the resident obs
    (dense 294->128->64->5 on MFMA, epsilon-greedy, writes actions[:, 0]):
    HBM-bound on reading the obs (E * W*W*6 f32); (2) the train_jax.py:42-64
    loop shape per step: act -> step + obs -> replay add_many (capacity
    MEMORY_SIZE), without the learner (train_loop_bench has it).
    `precision` is the loop's (f32: the reference's nets); both acts are
    timed alone, and the f32 act from the policy code (drl_qnet_act_code,
    128 B per env read instead of 1,176).  `input` is the loop act's."""
    from dronerl_amd.dqn import QNetwork, ReplayBuffer
    E = env.num_envs
    D = obs[0].numel()
    net = QNetwork(D, (128, 64), device=env.device, generator=torch.Generator().manual_seed(0), precision=precision)
    rb = ReplayBuffer(MEMORY_SIZE, D, env.device)
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
    lnet = net
    if input == "code":  # the step writes drone 0's policy code alone; the replay holds code rows
        lnet = QNetwork(D, (128, 64), device=env.device, generator=torch.Generator().manual_seed(0),
                        precision="f32", input="code")
        bufs = [env.new_code(), env.new_code()]
        env.get_code(out=bufs[0])
        rb = ReplayBuffer(MEMORY_SIZE, D, env.device, code_radius=env.params.window_radius)
    ev[2].record(stream)
    for t in range(steps):
        cur, nxt = bufs[t & 1], bufs[(t + 1) & 1]
        a = actions[t % actions.shape[0]]
        if input == "code":
            lnet.act(cur, 0.1, seed=1, step=t, actions=a)
            env.step(a, rewards=rewards, dones=dones, code=nxt)
        else:
            lnet.act(cur.reshape(E, -1), 0.1, seed=1, step=t, actions=a)
            env.step(a, obs_k=1, rewards=rewards, dones=dones, obs=nxt)
        rb.add_many(cur, a, rewards, nxt, dones)
    ev[3].record(stream)
    torch.cuda.synchronize()
    env.check_errors()
    lnet.check_errors()  # the f32 acts flag operands outside fp16's split range only through the net
    # the f32 act from the policy code of the same state
    act_code = act_code_rl = None
    W = env.layout.obs_window
    if W in (5, 7, 9):
        cnet = lnet if input == "code" else QNetwork(D, (128, 64), device=env.device,
                                                     generator=torch.Generator().manual_seed(0),
                                                     precision="f32", input="code")
        code = env.new_code()
        env.get_obs(1, out=obs, code=code)
        for t in range(warmup):
            cnet.act(code, 0.1, seed=1, step=t, actions=a0)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for t in range(steps):
            cnet.act(code, 0.1, seed=1, step=t, actions=a0)
        c1.record(stream)
        torch.cuda.synchronize()
        act_code = c0.elapsed_time(c1) / 1e3 / steps
        cnet.check_errors()
        act_code_rl = act_code_roofline(E, W, act_code)
    # the act in the other precision
    other = "bf16" if precision == "f32" else "f32"
    net32 = QNetwork(D, (128, 64), device=env.device, generator=torch.Generator().manual_seed(0), precision=other)
    for t in range(warmup):
        net32.act(flat, 0.1, seed=1, step=t, actions=a0)
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record(stream)
    for t in range(steps):
        net32.act(flat, 0.1, seed=1, step=t, actions=a0)
    f1.record(stream)
    torch.cuda.synchronize()
    act_o = f0.elapsed_time(f1) / 1e3 / steps
    act_s = ev[0].elapsed_time(ev[1]) / 1e3 / steps
    loop_s = ev[2].elapsed_time(ev[3]) / 1e3 / steps
    read = E * D * 4
    t = {"bf16": (act_o, act_s), "f32": (act_s, act_o)}[other]
    rl = lambda s: {"bound": "hbm", "achieved": read / s / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",  # noqa: E731
                    "frac": read / s / 1e9 / PEAK_HBM_GBS, "algorithmic_bytes_per_env": D * 4 + 4}
    return {"net": f"dense {D}->128->64->5", "precision": precision,
            "act_f32_us": t[1] * 1e6, "act_f32_roofline": rl(t[1]),
            "act_f32_note": "precision='f32' (DRL_QNET_F32): fp16 hi/lo split operands, 3 MFMAs per product tile, "
                            "Q to f32 rounding (the reference's f32 nets)",
            "act_bf16_us": t[0] * 1e6, "act_bf16_roofline": rl(t[0]),
            "act_bf16_note": "precision='bf16': bf16 MFMA operands, f32 accumulate (a labelled extra; narrower than "
                             "the reference)",
            "act_code_f32_us": None if act_code is None else act_code * 1e6,
            "act_code_roofline": act_code_rl,
            "act_code_note": "f32 act from drone 0's policy code (drl_qnet_act_code; the step writes it beside the "
                             "observation): inputs exact in fp16, 2 MFMAs per layer-0 product tile, Q to 1e-5 of "
                             "the f32 forward",
            "loop_us_per_step": loop_s * 1e6, "loop_env_steps_per_s": E / loop_s,
            "loop": (f"act(code_t, f32) -> step + drone 0 policy code -> replay add_many(code_t, a, r, "
                     f"code_t+1, done) of code rows, capacity {MEMORY_SIZE}; no learner (train_loop has it)")
                    if input == "code" else
                    (f"act(obs_t, {precision}) -> step + obs(K=1) -> replay add_many(obs_t, a, r, obs_t+1, done), "
                     f"capacity {MEMORY_SIZE}; no learner (train_loop has it)")}


MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md; the 16x16x32 f16 form: 16 cycles)


def act_code_flops(E: int, W: int, hidden=(128, 64), n_actions: int = 5):
    """FLOPs of one drl_qnet_act_code launch over E envs (W x W window, 6
    channels per cell; jax dqn.py:47-63's dense net).  Returns (executed,
    algorithmic): executed = the v_mfma_f32_16x16x32_f16 instructions the
    kernel issues (2*16*16*32 FLOPs each) per 16-env tile -- layer 0: its
    K-slices (6 slots per cell of each lane group's ceil(W*W/4) cells + the
    bias slot, 8 per slice, even count) x (h0/16) unit tiles x 2 (hi and lo
    weights; the inputs are exact in fp16); each later layer: (h_prev/32)
    K-slices x (h/16) tiles x 3 (hi*hi, hi*lo, lo*hi of the f32 split);
    algorithmic = the f32 net's 2 * E * sum(in*out)."""
    cpg = (W * W + 3) // 4
    kp0 = -(-(6 * cpg + 1) // 8)
    kp0 += kp0 % 2
    sizes = [W * W * 6, *hidden, n_actions]
    per_tile = kp0 * (hidden[0] // 16) * 2
    for i in range(1, len(sizes) - 1):
        per_tile += (sizes[i] // 32) * (-(-sizes[i + 1] // 16)) * 3
    tiles = -(-E // 16)
    executed = tiles * per_tile * 2 * 16 * 16 * 32
    algorithmic = 2 * E * sum(sizes[i] * sizes[i + 1] for i in range(len(sizes) - 1))
    return executed, algorithmic, per_tile


def act_code_roofline(E: int, W: int, launch_s: float):
    """SURVEY.md §8 F1's separate roofline for the MFMA consumer: the code act
    is matrix work (bound "mfma"): executed MFMA FLOPs per launch / its average
    launch duration (HIP events) against the dense f16 MFMA peak."""
    ex, alg, per_tile = act_code_flops(E, W)
    achieved = ex / launch_s / 1e12
    return {"bound": "mfma", "achieved": achieved, "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / MFMA_PEAK_TFLOPS, "mfma_flops_per_launch": ex, "mfma_per_16env_tile": per_tile,
            "algorithmic_f32_flops_per_launch": alg, "avg_launch_us": launch_s * 1e6,
            "note": "executed v_mfma_f32_16x16x32_f16 FLOPs (f32 numerics as fp16 hi/lo pieces: 2 MFMAs per layer-0 "
                    "product tile, 3 per later-layer tile) / average launch (HIP events); "
                    "algorithmic_f32_flops_per_launch is the plain f32 net's 2*E*sum(in*out)"}


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
                         "note": "same per-env-step algorithmic read bytes R as drl_step (SURVEY.md §8 D3); the "
                                 "state is read and written once per launch, so HBM traffic per step is lower"}}


# train_jax.py:351 --memory_size: the replay capacity of the train loops
MEMORY_SIZE = 100_000

# diagnostic: the train loop's step with streaming observation stores (A/B of
# env.step()'s store mode where the act kernel reads the observation next)
LOOP_OBS_STREAM = {"0": False, "1": True}.get(os.environ.get("DRL_LOOP_OBS_STREAM", ""))


class TrainSegment:
    """One segment of the train_jax.py:38-113 scan loop (C5:
    "multi-step loop, hipGraph of step+obs+act"): per step, synthetic actions
    for every drone, the epsilon-greedy DQN action for drone 0 (dense
    294->128->64->5, epsilon read from the learner's device counter), step +
    obs(K=1), replay add_many of the drone-0 transition into the reference's
    100,000-slot memory (train_jax.py:173, --memory_size), and the learner
    block (:68-98, drl_dqn_train: sample 8 rows + train_step + Adam, the target
    update every 10 steps, the epsilon decay every 5, step + 1); after `seg`
    steps a reset of every env (reset_env_every, train_jax.py:101-113) and its
    first observation.  learn=False drops the learner (epsilon fixed at 0.1).

    fused=True: the synthetic actions of drones 1..N-1 are written by the act
    launch itself (drl_qnet_act_synth), one kernel fewer per step with the
    same action rows.

    parallel=True: the replay add (and, unfused, the synthetic actions) run on
    side streams, joined to the act -> step chain by events; so does the
    respawn-candidate refill (env.step()'s cadence, launched on its own branch
    after the step it follows: it overlaps the next act, and the next step
    waits for it).  The learner follows the add of its step on the main
    stream without waiting for the add of its step (it reads that step's
    transitions from the step's buffers: drl_dqn_train_fresh), and the next
    act follows the learner (it acts with the updated net).  Observations, actions,
    rewards and dones rotate through 3 buffers, so step t only waits for the
    replay add of step t-2 and the actions of step t are drawn while step t-1
    runs.  parallel=False issues the same calls in the same order on one
    stream with 2 buffers; both leave identical state and replay contents
    (tests/test_gpu_parity.py::test_train_segment_parallel_matches_serial)."""

    def __init__(self, env, seg: int, parallel: bool = False, net=None, rb=None, fused: bool = True,
                 precision: str = "f32", input: str = "obs", learn: bool = True, capacity: int = MEMORY_SIZE,
                 hp=None, fuse_replay=None, refill_branch: bool = False, synth_branch: bool = False,
                 synth_in_step=None):
        from dronerl_amd.dqn import DQNHParams, DQNLearner, QNetwork, ReplayBuffer
        E, N, dev = env.num_envs, env.n_drones, env.device
        W = env.layout.obs_window
        D = W * W * 6
        self.env, self.seg, self.parallel, self.E = env, seg, parallel, E
        # input "code": the step writes drone 0's policy code instead of the
        # f32 observation (128 B per env instead of 1,176), the act reads it
        # (f32 nets; Q to 1e-5 of the f32 forward) and the replay buffer
        # stores code rows, decoding the rows it samples to the observation
        self.input = input
        self.fused = fused
        # fuse_replay (code input, one stream; the default there): the step lands its drone-0 transitions in
        # the ring itself (drl_step_code_replay) -- no replay-add launch, and the code rows are not read back
        if fuse_replay is None:
            fuse_replay = input == "code" and not parallel
        if fuse_replay and (input != "code" or parallel):
            raise ValueError("fuse_replay needs input='code' and parallel=False")
        self.fuse_replay = fuse_replay
        # synth_in_step (with fuse_replay; the default there): the fused step draws drones 1..N-1's synthetic
        # actions itself (drl_step_code_replay_synth) and the act writes drone 0's column only -- the act no
        # longer computes and writes N - 1 columns that the step reads back
        if synth_in_step is None:
            synth_in_step = fuse_replay and not synth_branch
        if synth_in_step and not fuse_replay:
            raise ValueError("synth_in_step needs the fused replay step")
        self.synth_in_step = synth_in_step
        self.refill_branch = refill_branch  # (one stream: the refill on its own graph branch, see run)
        # synth_branch (one stream, unfused): the synthetic actions of step t + 1 on their own graph branch,
        # forked after step t and joined before act t + 1, so they run beside learner t (see run)
        if synth_branch and (fused or parallel):
            raise ValueError("synth_branch needs fused=False and parallel=False")
        self.synth_branch = synth_branch
        # parallel branches need 3 rotating buffers (see above); on one stream 2
        # suffice, and the third 77 MB observation buffer costs MALL hits (C3
        # loop 79.4 vs 74.4 us per step)
        self.NB = 3 if parallel else 2
        self.net = net or QNetwork(D, (128, 64), device=dev, generator=torch.Generator().manual_seed(0),
                                   precision=precision, input=input)
        self.rb = rb or ReplayBuffer(capacity, D, dev, code_radius=env.params.window_radius if input == "code" else 0)
        self.learner = DQNLearner(self.net, hp or DQNHParams(), generator=torch.Generator().manual_seed(1)) \
            if learn else None
        self.acts = [torch.empty((E, N), dtype=torch.int32, device=dev) for _ in range(self.NB)]
        self.rewards = [torch.empty((E, N), dtype=torch.float32, device=dev) for _ in range(self.NB)]
        self.dones = [torch.empty((E, N), dtype=torch.uint8, device=dev) for _ in range(self.NB)]
        if input == "code":
            self.obs = self.code = [env.new_code() for _ in range(self.NB)]
        else:
            self.obs = [torch.empty((E, 1, W, W, 6), dtype=torch.float32, device=dev) for _ in range(self.NB)]
        self._first_obs()
        self.s_syn, self.s_rep, self.s_ref = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def _first_obs(self):
        if self.input == "code":
            self.env.get_code(out=self.code[0])
        else:
            self.env.get_obs(1, out=self.obs[0])

    def _synth(self, t):
        self.env.synth_actions(seed=2024, step=t, out=self.acts[t % self.NB])

    def _act_step(self, t, before_step=None):
        b, nb = t % self.NB, (t + 1) % self.NB
        x = self.code[b] if self.input == "code" else self.obs[b].reshape(self.E, -1)
        eps = self.learner.epsilon if self.learner is not None else 0.1
        self.net.act(x, eps, seed=7, step=t, env_offset=self.env.env_offset,
                     actions=self.acts[b], synth=(2024, t) if self.fused and not self.synth_in_step else None)
        if before_step is not None:  # (parallel: the refill branch joins here)
            before_step()
        if self.fuse_replay:
            self.env.step(self.acts[b], rewards=self.rewards[b], dones=self.dones[b], code=self.code[nb],
                          replay=self.rb, replay_obs=self.code[b], synth=(2024, t) if self.synth_in_step else None)
        elif self.input == "code":
            self.env.step(self.acts[b], rewards=self.rewards[b], dones=self.dones[b], code=self.code[nb])
        else:
            self.env.step(self.acts[b], obs_k=1, rewards=self.rewards[b], dones=self.dones[b], obs=self.obs[nb],
                          obs_stream=LOOP_OBS_STREAM)  # None: env.step()'s default

    def _replay(self, t):
        if self.fuse_replay:  # the step of _act_step(t) has added them (drl_step_code_replay)
            return self.rb.last_batch
        b, nb = t % self.NB, (t + 1) % self.NB
        return self.rb.add_many(self.obs[b], self.acts[b], self.rewards[b], self.obs[nb], self.dones[b])

    def _learn(self, fresh=None):
        if self.learner is not None:
            self.learner.train(self.rb, fresh=fresh)

    def run(self):
        main = torch.cuda.current_stream(self.env.device)
        if not self.parallel and self.refill_branch and self.env.refill_every > 0:
            # (A/B, off by default) one stream, except the respawn-candidate refill (env.step()'s cadence): it
            # only reads and writes the MT rows, which the learner and the next act do not touch, so it can run
            # on its own branch after the step it follows, the next step waiting for it.  Measured
            # (gpurun_out r06i, tools/loop_refill_ab.sh): C3 71.6 / 71.1 against 70.2 / 69.6 us per step inline,
            # C5 248.7 / 248.5 against 248.6 / 248.0 -- the refill's HBM stream slows the learner's hand-offs
            # as much as the overlap saves
            every = self.env.refill_every
            self.env.refill_every = 0
            since = self.env._since_refill
            ev_ref = None
            try:
                for t in range(self.seg):
                    if not self.fused:
                        self._synth(t)
                    join = (lambda e=ev_ref: main.wait_event(e)) if ev_ref is not None else None
                    self._act_step(t, before_step=join)
                    ev_ref = None
                    since += 1
                    if since >= every:
                        since = 0
                        ev_step = torch.cuda.Event()
                        ev_step.record(main)
                        with torch.cuda.stream(self.s_ref):
                            self.s_ref.wait_event(ev_step)
                            self.env.refill()
                            ev_ref = torch.cuda.Event()
                            ev_ref.record(self.s_ref)
                    self._replay(t)
                    self._learn()
                main.wait_stream(self.s_ref)
            finally:
                self.env.refill_every = every
                self.env._since_refill = since
        elif not self.parallel and self.synth_branch:
            # acts[(t + 1) % 2] was last read by step t - 1, which precedes the fork after step t
            def fork(t):
                ev = torch.cuda.Event()
                ev.record(main)
                with torch.cuda.stream(self.s_syn):
                    self.s_syn.wait_event(ev)
                    self._synth(t)
                    done = torch.cuda.Event()
                    done.record(self.s_syn)
                return done
            ev_syn = fork(0)
            for t in range(self.seg):
                main.wait_event(ev_syn)  # (the act writes column 0 of the same rows)
                self._act_step(t)
                self._replay(t)
                if t + 1 < self.seg:
                    ev_syn = fork(t + 1)
                self._learn()
            main.wait_stream(self.s_syn)
        elif not self.parallel:
            for t in range(self.seg):
                if not self.fused:
                    self._synth(t)
                self._act_step(t)
                self._replay(t)
                self._learn()
        else:
            ev_syn = [torch.cuda.Event() for _ in range(self.seg)]
            ev_step = [torch.cuda.Event() for _ in range(self.seg)]
            ev_rep = [torch.cuda.Event() for _ in range(self.seg)]
            ev_ref = None
            every = self.env.refill_every
            self.env.refill_every = 0  # (the refills below, on their own branch)
            since = self.env._since_refill
            try:  # (a capture that raises must not leave the env with refills off: ADVICE r3)
                self.s_syn.wait_stream(main)
                self.s_rep.wait_stream(main)
                for t in range(self.seg):
                    if not self.fused:
                        with torch.cuda.stream(self.s_syn):
                            if t >= self.NB:  # acts[t % 3] was last read by the replay add of step t-3
                                self.s_syn.wait_event(ev_rep[t - self.NB])
                            self._synth(t)
                            ev_syn[t].record(self.s_syn)
                        main.wait_event(ev_syn[t])
                    elif t >= self.NB:  # the act writes acts[t % 3], read by the replay add of step t-3
                        main.wait_event(ev_rep[t - self.NB])
                    if t >= 2:  # step t overwrites obs[(t+1) % 3], read by the replay add of step t-2
                        main.wait_event(ev_rep[t - 2])
                    join = (lambda e=ev_ref: main.wait_event(e)) if ev_ref is not None else None
                    self._act_step(t, before_step=join)
                    ev_ref = None
                    ev_step[t].record(main)
                    since += 1
                    if every > 0 and since >= every:
                        since = 0
                        with torch.cuda.stream(self.s_ref):
                            self.s_ref.wait_event(ev_step[t])
                            self.env.refill()
                            ev_ref = torch.cuda.Event()
                            ev_ref.record(self.s_ref)
                    with torch.cuda.stream(self.s_rep):
                        self.s_rep.wait_event(ev_step[t])
                        batch = self._replay(t)
                        ev_rep[t].record(self.s_rep)
                    if self.learner is not None:
                        # the learner reads step t's transitions from the step's own buffers (fresh), so it
                        # overlaps the add of step t; the ring rows of step t - 1 must have landed
                        if t >= 1:
                            main.wait_event(ev_rep[t - 1])
                        self._learn(fresh=batch)
                main.wait_stream(self.s_syn)
                main.wait_stream(self.s_rep)
                main.wait_stream(self.s_ref)
            finally:
                self.env.refill_every = every
                self.env._since_refill = since
        self.env.reset(seed=None)
        self._first_obs()


def train_loop_bench(env, reps: int, seg: int = 100, parallel: bool = False, fused: bool = True,
                     precision: str = "f32", input: str = "obs", learn: bool = True, refill_branch: bool = False,
                     synth_branch: bool = False, synth_in_step=None):
    """TrainSegment captured once as a HIP graph (no host work per step) and
    replayed.  The host-side counters (action stream step, exploration draws,
    replay cursor) are baked into the capture, so replays repeat them: the
    work per step is the same, the action stream repeats every segment.  The
    learner's counters (step, Adam count, epsilon, sampled rows) live on the
    device and continue across replays."""
    dev = env.device
    loop = TrainSegment(env, seg, parallel=parallel, fused=fused, precision=precision, input=input, learn=learn,
                        refill_branch=refill_branch, synth_branch=synth_branch, synth_in_step=synth_in_step)
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
    loop.net.check_errors()  # (an f32 act's range flag lives in the net)
    dt = e0.elapsed_time(e1) / 1e3
    E = env.num_envs
    lr = loop.learner
    learner = None
    if lr is not None:
        c = lr.counters()
        # the learner alone, back to back on the loop's filled replay (HIP events around 50 launches; its
        # device counters advance, nothing else is touched)
        torch.cuda.synchronize(dev)
        l0, l1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        l0.record()
        for _ in range(50):
            lr.train(loop.rb)
        l1.record()
        torch.cuda.synchronize(dev)
        lr.check_errors()
        learner_us = l0.elapsed_time(l1) * 1e3 / 50
        c = lr.counters()
        learner = {"us_per_launch_alone": learner_us, "batch": lr.hp.batch, "learning_rate": lr.hp.learning_rate, "gamma": lr.hp.gamma,
                   "tau": lr.hp.tau, "target_update_interval": lr.hp.target_update_interval,
                   "epsilon_decay_every": lr.hp.epsilon_decay_every, "epsilon_decay": lr.hp.decay(),
                   "replay_capacity": loop.rb.capacity, "steps_taken": c["step"], "adam_steps": c["count"],
                   "epsilon_after": c["epsilon"], "last_loss": c["loss"],
                   "note": "drl_dqn_train every step: sample + train_step (TD-MSE backward) + optax Adam, target "
                           "update and epsilon decay on the device (train_jax.py:68-98); us_per_launch_alone: 50 "
                           "launches back to back after the loop (latency-bound: DESIGN.md section 4 has the "
                           "phase times)",
                   "parallelism": "one learner per rank, on that rank's env shard and replay (replicas). The "
                                  "reference's sharded jit run trains one global learner: that mode is "
                                  "dronerl_amd.global_learner (each rank's image of the one global ring, the "
                                  "sampled rows gathered from their owners, ~2 KB all_gather per step; bit-exact "
                                  "against one learner in tests/test_gpu_multirank.py), not timed here "
                                  "(DESIGN.md section 6)"}
    branches = (("replay add_many" if fused else "synthetic actions and replay add_many") +
                " on parallel graph branches, 3 rotating buffers" if parallel else
                "one stream, the refill on its own graph branch" if loop.refill_branch else "one stream") + \
        ("; drones 1..N-1's synthetic actions drawn inside the step launch (drl_step_code_replay_synth)"
         if loop.synth_in_step else "; synthetic actions inside the act launch" if fused else
         "; synthetic actions on their own graph branch beside the learner" if loop.synth_branch else "") + \
        ("; the replay add inside the step launch (drl_step_code_replay)" if loop.fuse_replay else "")
    return {"env_steps_per_s": E * seg * reps / dt, "us_per_step": dt / (seg * reps) * 1e6,
            "segments": reps, "steps_per_segment": seg, "precision": precision, "input": input,
            "learner": learner,
            "loop": f"hipGraph of {seg} x [synth actions -> qnet act (drone 0, {precision}, input {input}, device "
                    f"epsilon) -> step + {'drone 0 policy code' if input == 'code' else 'obs(K=1)'} -> "
                    f"replay add_many{' (code rows)' if input == 'code' else ''} into {loop.rb.capacity} slots"
                    f"{' -> learner (drl_dqn_train)' if learn else ''}] + reset + obs, replayed {reps}x "
                    f"({branches}{'' if learn else '; learner not included'})"}


def loop_input(args, env) -> str:
    """--loop-input auto: the policy code wherever a code-input net applies
    (f32 precision, a 5x5, 7x7 or 9x9 window)."""
    if args.loop_input != "auto":
        return args.loop_input
    return "code" if args.loop_precision == "f32" and env.layout.obs_window in (5, 7, 9) else "obs"


# refill cycles of untimed steps after the reset, before the warm-up: the
# refills measured there (all but the first two) price the timed region's
# pro-rated refill share at short step counts (tools/refill_time.py: the
# steady state needs a few cycles after a reset)
PRE_ROLL_CYCLES = 8


def refill_plan(pre: int, warmup: int, steps: int, every: int):
    """env.step()'s refill cadence over one bench run: drl_refill follows
    global step s when (s + 1) % every == 0, counting from the first pre-roll
    step.  Returns the timed steps a refill follows and the share of a refill
    still to charge the timed region, steps / every - (refills inside it):
    every timed step then carries exactly 1/every of a refill whatever the
    step count (a 20-step window holds no refill at every = 32; a 1000-step
    one holds 31 and is charged 0.25 more)."""
    if every <= 0:
        return [], 0.0
    first = pre + warmup
    inside = [s for s in range(first, first + steps) if (s + 1) % every == 0]
    return inside, steps / every - len(inside)


class StepRunner:
    """The timed loop of one config: drl_step_ex launches through a ctypes
    fast path (arguments built once; only the actions pointer moves), with
    drl_refill at env.step()'s cadence bracketed by HIP events on the launch
    stream, so the step kernel's average duration and the refills' can be
    told apart.  Actions are synthetic uniform {0..4} (counter hash),
    generated before timing and resident in HBM."""

    def __init__(self, env, K: int, n_actions: int, obs_stream: bool):
        from dronerl_amd._native import DRL_STEP_OBS_STREAM, lib
        E, N, dev = env.num_envs, env.n_drones, env.device
        self.env, self.K, self.E = env, K, E
        self.L = lib()
        self.stream = torch.cuda.current_stream(dev)
        self.actions = torch.empty((n_actions, E, N), dtype=torch.int32, device=dev)
        for t in range(n_actions):
            env.synth_actions(seed=2024, step=t, out=self.actions[t])
        W = env.layout.obs_window
        self.rewards = torch.empty((E, N), dtype=torch.float32, device=dev)
        self.dones = torch.empty((E, N), dtype=torch.uint8, device=dev)
        self.obs = torch.empty((E, max(K, 1), W, W, 6), dtype=torch.float32, device=dev)
        self._cp = ctypes.byref(env._cp)
        self._st = env.state.c()
        self._sp = ctypes.byref(self._st)
        self._a = [ctypes.c_void_p(self.actions[t].data_ptr()) for t in range(n_actions)]
        self._r, self._d, self._o = (ctypes.c_void_p(x.data_ptr()) for x in (self.rewards, self.dones, self.obs))
        if K == 0:
            self._o = None
        self._e = ctypes.c_void_p(env.err.data_ptr())
        self._s = ctypes.c_void_p(self.stream.cuda_stream)
        self.flag_stream = DRL_STEP_OBS_STREAM
        self.obs_stream = obs_stream
        self.every = env.refill_every
        self.s = 0  # global step counter (refill cadence)
        self.refill_ev = []  # (start, end, timed) events of every refill

    def step(self, timed: bool):
        t = self.s % len(self._a)
        flags = self.flag_stream if self.obs_stream else 0
        rc = self.L.drl_step_ex(self._cp, self._sp, self._a[t], self._r, self._d, self._o, self.K, self._e, flags,
                                self._s)
        if rc:
            raise RuntimeError(self.L.drl_last_error().decode())
        if self.every > 0 and (self.s + 1) % self.every == 0:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(self.stream)
            rc = self.L.drl_refill(self._cp, self._sp, self._s)
            if rc:
                raise RuntimeError(self.L.drl_last_error().decode())
            ev[1].record(self.stream)
            self.refill_ev.append(ev + (timed,))
        self.s += 1

    def run(self, steps: int, warmup: int, world: int, pre: int = 0):
        """pre + warmup untimed steps, then `steps` timed ones bracketed by a
        barrier + synchronize on both sides, max over ranks.  The region's
        time is the HIP-event time on the launch stream from its first launch
        to its last (the host's wall clock of the same region, which adds the
        queue's start and drain latency, ~1 us per step over 20 steps and
        0.02 over 1000, is reported as wall_ms_per_step).  The value charges
        the timed region steps/every refills (refill_plan)."""
        for _ in range(pre + warmup):
            self.step(False)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        n_before = len(self.refill_ev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(self.stream)
        for _ in range(steps):
            self.step(True)
        ev1.record(self.stream)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        self.env.check_errors()
        wall_max = max_over_ranks(wall, world)
        inside = [e for e in self.refill_ev[n_before:] if e[2]]
        plan, charge = refill_plan(0, self.s - steps, steps, self.every)
        assert len(plan) == len(inside), (plan, len(inside))
        ref_in_ms = sum(a.elapsed_time(b) for a, b, _ in inside)
        # the refill's average launch: every one measured except the first two
        # after the reset (the first fills the empty rings; the rings of all
        # envs then cross block ends in step, so the next few refills are
        # lighter than the steady state a long run sees -- hence the pre-roll
        # of PRE_ROLL_CYCLES refill cycles)
        all_ms = [a.elapsed_time(b) for a, b, _ in self.refill_ev]
        use = all_ms[2:] if len(all_ms) > 2 else all_ms[-1:]
        refill_avg_s = max_over_ranks(sum(use) / len(use) / 1e3 if use else 0.0, world)
        region_s = max_over_ranks(ev0.elapsed_time(ev1) / 1e3, world)
        charged = region_s + charge * refill_avg_s
        launch_s = (ev0.elapsed_time(ev1) - ref_in_ms) / 1e3 / steps  # drl_step kernel, on this stream
        return {"value": self.E * world * steps / charged, "ms_per_step": charged / steps * 1e3,
                "wall_ms_per_step": wall_max / steps * 1e3, "launch_s": launch_s,
                "refill": {"every": self.every, "launches_in_region": len(inside),
                           "launches_measured": len(all_ms), "avg_launch_us": refill_avg_s * 1e6,
                           "per_step_us": refill_avg_s / self.every * 1e6 if self.every > 0 else 0.0,
                           "charged_launches": steps / self.every if self.every > 0 else 0.0,
                           "prorated_launches": charge,
                           "note": "env.step()'s cadence (a refill after every `every`-th step, counted from the "
                                   "pre-roll); the timed region is charged exactly steps/every refills: the ones "
                                   "inside it plus prorated_launches x avg_launch_us (HIP events; the pre-roll's "
                                   "first refill excluded), so value and ms_per_step carry the refill share at any "
                                   "step count"}}


def measure_copy_peak(dev, nbytes: int = 2 << 30, reps: int = 8):
    """the measured copy-kernel rate beside the 8 TB/s spec
    (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy).  drl_hbm_probe is that
    plain float4 copy (one 16-B element per lane, a grid over the buffer),
    run over two 2-GiB buffers (past the 256-MiB Infinity Cache); each launch
    is timed alone with HIP events on the launch stream and the best one is
    the rate: copy = GB/s of bytes read + written, read = a read-only pass."""
    from dronerl_amd._native import lib
    L = lib()
    a = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream(dev)
    out = {}
    for name, mode, mult in (("copy", 0, 2), ("read", 1, 1)):
        run = lambda: L.drl_hbm_probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),  # noqa: E731
                                      nbytes, mode, ctypes.c_void_p(st.cuda_stream))
        if run():
            raise RuntimeError(L.drl_last_error().decode())
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in ev:
            e0.record(st)
            run()
            e1.record(st)
        torch.cuda.synchronize(dev)
        best = min(e0.elapsed_time(e1) for e0, e1 in ev) / 1e3
        out[name] = mult * nbytes / best / 1e9
    del a, b
    torch.cuda.empty_cache()
    return {"copy_GBs": out["copy"], "read_GBs": out["read"],
            "note": f"in-run probe: drl_hbm_probe, a plain float4 copy (read + write bytes) and a read-only pass "
                    f"over {nbytes >> 20} MiB buffers on this GPU, best of {reps} launches each"}


def measured_peak(peak_measured, *rates):
    """The measured HBM peak the *_vs_measured_peak fractions divide by: the
    best of the probe's copy and read rates and of any kernel's own measured
    traffic rate (a kernel that out-runs the probe sets the peak), so every
    such fraction is <= 1 (tests/test_bench_contract.py)."""
    cands = [("drl_hbm_probe copy", peak_measured["copy_GBs"]), ("drl_hbm_probe read", peak_measured["read_GBs"])]
    cands += [(name, r) for name, r in rates if r]
    return max(cands, key=lambda c: c[1])


def roofline(E, R, Wb, launch_s, refill, traffic, G=None, peak_measured=None):
    """SURVEY.md §8 D3 roofline of the dominant kernel (drl_step_kernel):
    achieved = E * R (algorithmic read bytes per env-step) / its average
    launch duration (HIP events on the launch stream).  `traffic` = measured
    HBM bytes per launch (PMC); frac_measured = traffic / launch / peak, the
    fraction of the HBM peak the kernel actually moves (<= 1 by construction).
    frac_ceiling = R / ((R - G^2/2) + (W - G^2)): the frac of a kernel that
    moves only its obligatory bytes at the spec peak -- the ground as stored
    (two cells per byte, ABI 8: R counts G^2 but G^2/2 are read), the outputs
    every step must write (observation, rewards, dones, records), no ground
    write-back (the survey's W counts all G^2 ground bytes; a step writes only
    the changed cells).  It bounds frac for any launch at or below the spec
    peak, and exceeds 1 where R's ground count exceeds the stored bytes (C5).
    peak_measured: the in-run probe (measured_peak: frac_vs_measured_peak =
    achieved / the best measured rate).  with_refill adds the refill share per
    step."""
    achieved = E * R / launch_s / 1e9
    ceiling = R / (R - (G * G - (G * G + 1) // 2 if G else 0) + Wb - (G * G if G else 0))
    out = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": "drl_step_kernel",
           "avg_launch_us": launch_s * 1e6, "algorithmic_read_bytes_per_env_step": R,
           "algorithmic_write_bytes_per_env_step": Wb, "frac_ceiling": ceiling,
           "note": "frac counts SURVEY.md §8 D3's read bytes R only (achieved = E*R / avg drl_step launch); "
                   "frac_ceiling = R/((R - G^2/2) + (W - G^2)) bounds it (the obligatory bytes -- the packed ground, "
                   "the outputs -- moved at the spec peak, no ground write-back). traffic = measured HBM bytes per drl_step launch (2*FETCH_SIZE + "
                   "WRITE_SIZE), frac_measured = traffic / avg launch / peak"}
    kernel_rate = traffic["drl_step_kernel"]["bytes_per_launch"] / launch_s / 1e9 if traffic else None
    if peak_measured:
        src, peak = measured_peak(peak_measured, ("drl_step_kernel traffic", kernel_rate))
        out["peak_measured"] = peak
        out["peak_measured_source"] = src
        out["frac_vs_measured_peak"] = achieved / peak
        out["peak_measured_detail"] = peak_measured
    per_step_s = launch_s + refill["per_step_us"] / 1e6
    out["with_refill"] = {"us_per_step": per_step_s * 1e6, "achieved": E * R / per_step_s / 1e9,
                          "frac": E * R / per_step_s / 1e9 / PEAK_HBM_GBS}
    if traffic:
        st = traffic["drl_step_kernel"]
        out["traffic"] = st["bytes_per_launch"]
        out["frac_measured"] = st["bytes_per_launch"] / launch_s / 1e9 / PEAK_HBM_GBS
        if peak_measured:
            out["frac_measured_vs_measured_peak"] = kernel_rate / out["peak_measured"]
        out["traffic_detail"] = dict(st, source=traffic.get("source"), envs=traffic.get("envs"))
        rf = traffic.get("drl_refill_list_kernel") or traffic.get("drl_refill_kernel")
        if rf and refill["every"] > 0:
            per_step_b = st["bytes_per_launch"] + rf["bytes_per_launch"] / refill["every"]
            out["with_refill"].update({"traffic_per_step": per_step_b,
                                       "frac_measured": per_step_b / per_step_s / 1e9 / PEAK_HBM_GBS,
                                       "refill_traffic_per_launch": rf["bytes_per_launch"],
                                       "refill_read_bytes_per_env": rf["read_bytes_per_env"],
                                       "refill_write_bytes_per_env": rf["write_bytes_per_env"]})
    return out


def make_env(cfg: str, envs: int, rank: int, dev):
    from dronerl_amd import BatchedDeliveryDrones, EnvParams
    G, N, E, K = CONFIGS[cfg]
    E = envs or E
    env = BatchedDeliveryDrones(EnvParams(n_drones=N, grid_size=G), E, device=dev, env_offset=rank * E)
    env.reset(seed=0)
    return env, G, N, E, K


def pmc_child(args):
    """--pmc-child: the step loops the rocprofv3 counter passes of
    measure_traffic profile (no timing, no extras); prints each config's
    launch grid sizes (threads) so the parent can attribute the rows."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    grids = {}
    for name in args.pmc_child.split(","):
        envs = args.c5_envs if name == "c5" and args.config != "c5" else args.envs
        env, G, N, E, K = make_env(name, envs, 0, dev)
        if args.obs_k >= 0 and name == args.config:
            K = args.obs_k
        stream = args.obs_stream or (env.default_obs_stream and not args.obs_cached)
        run = StepRunner(env, K, 8, stream)
        run.run(args.steps, args.warmup, 1, pre=PRE_ROLL_CYCLES * env.refill_every)
        P = env.layout.step_group_lanes
        grids[name] = {"envs": E, "step_grid": -(-E // (64 // P)) * 64, "refill_grid": -(-E // 4) * 64,
                       "refill_list_grid": -(-E // 32) * 512}
        del run, env
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    print(json.dumps({"pmc_child": grids}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=0, help="override envs per GPU")
    ap.add_argument("--c5-envs", type=int, default=CONFIGS["c5"][2],
                    help="envs per GPU of the north-star sub-record (C5: 64x64 grid, 32 drones; 131072 per GPU = "
                         "2^20 over 8 GPUs; 0 = skip)")
    ap.add_argument("--c5-steps", type=int, default=200, help="timed steps of the north-star sub-record (>= 200)")
    ap.add_argument("--strong-envs", type=int, default=65536,
                    help="whole-job envs of the strong-scaling sub-record at N > 1 ranks (BASELINE.json: "
                         "num_envs=65536 over 1/2/4/8 GPUs; 0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-reset-bench", action="store_true")
    ap.add_argument("--no-dqn", action="store_true", help="skip the DQN-consumer measurement (SURVEY.md §8 F1)")
    ap.add_argument("--loop-precision", default="f32", choices=("f32", "bf16"),
                    help="Q-network arithmetic of the DQN loops (f32: the reference's nets; bf16 reported beside)")
    ap.add_argument("--loop-input", default="auto", choices=("auto", "obs", "code"),
                    help="the DQN loops' act input: the f32 observation or drone 0's policy code (f32 nets, 5x5..9x9 "
                         "windows); auto = code where it applies")
    ap.add_argument("--rollout-chunk", type=int, default=100,
                    help="steps per drl_rollout launch for the rollout measurement (0 = skip)")
    ap.add_argument("--loop-segments", type=int, default=3,
                    help="train-loop graph replays (100 steps + reset each; 0 = skip)")
    ap.add_argument("--unfused-act", action="store_true",
                    help="train loop: synthetic actions as their own launch instead of inside the act launch")
    ap.add_argument("--parallel-loop", action="store_true",
                    help="train loop with the replay add (and unfused synth) on parallel graph branches (with the "
                         "f32 observation: slower, the step kernel fills every CU in one generation and co-running "
                         "kernels delay its waves)")
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
    ap.add_argument("--pmc-child", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args)
    if needs_launch(args):  # N ranks as a child job, before this process touches the GPU
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))

    north = args.c5_envs > 0 and args.config != "c5"
    names = [args.config] + (["c5"] if north else [])
    traffic_run = None
    if (not args.no_pmc_traffic and int(os.environ.get("RANK", "0")) == 0
            and os.environ.get("DRL_BENCH_PMC", "1") != "0"):
        traffic_run = measure_traffic(args, names)  # child processes, before this one touches the GPU

    rank, world, local = dist_init()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    dev = torch.device("cuda", local)
    env, G, N, E, K = make_env(args.config, args.envs, rank, dev)
    if args.obs_k >= 0:
        K = args.obs_k
    if not args.obs_stream and not args.obs_cached:  # env.step()'s default store mode
        args.obs_stream = env.default_obs_stream
    W = env.layout.obs_window
    R, Wb = algorithmic_bytes(G, N, K, W)

    # ---- the headline: setup rolls one refill cycle (steady-state rings),
    # then W warm-up and K timed steps
    runner = StepRunner(env, K, args.warmup + args.steps + 2 * env.refill_every, args.obs_stream)
    main_res = runner.run(args.steps, args.warmup, world, pre=PRE_ROLL_CYCLES * env.refill_every)
    actions, rewards, dones, obs, stream = runner.actions, runner.rewards, runner.dones, runner.obs, runner.stream

    def traffic_of(name):
        if traffic_run is not None and name in traffic_run:
            return traffic_run[name]
        t = load_traffic(name)
        if t is None:
            return None
        return {"drl_step_kernel": {"bytes_per_launch": t},
                "source": f"committed profiles/pmc_{name}.json (an earlier run; no rocprofv3 pass in this one)"}

    # ---- the other observation store mode, same steps
    other = None
    if args.cached_steps > 0 and K > 0:
        runner.obs_stream = not args.obs_stream
        nc = min(args.cached_steps, args.steps)
        o = runner.run(nc, min(args.warmup, 20), world)
        runner.obs_stream = args.obs_stream
        other = {"value": o["value"], "unit": "env-steps/s", "steps": nc, "ms_per_step": o["ms_per_step"],
                 "avg_launch_us": o["launch_s"] * 1e6, "frac": E * R / o["launch_s"] / 1e9 / PEAK_HBM_GBS,
                 "obs_stores": "cached" if args.obs_stream else "streaming",
                 "note": "the other observation store mode, same steps and results, refill share charged the same "
                         "way; `value` uses env.step()'s default (cached stores at 8 lanes per env, streaming at "
                         ">= 16: the faster one in the train loop, profiles/r02_store_mode/)"}

    # ---- strong scaling (BASELINE.json's metric as written: num_envs = 65536
    # over the job): the same config, strong_envs / world envs per rank
    strong = None
    if args.strong_envs > 0:
        if world == 1:
            strong = {"value": main_res["value"], "num_envs_total": E, "n_gpus": 1, "scaling": "strong",
                      "note": "one rank: the headline itself" + ("" if E == args.strong_envs else
                                                                 f" ({E} envs, not {args.strong_envs})")}
        else:
            Es = strong_split(args.strong_envs, world)
            env_s, _, _, _, _ = make_env(args.config, Es, rank, dev)
            run_s = StepRunner(env_s, K, args.warmup + args.steps + 2 * env_s.refill_every, args.obs_stream)
            rs = run_s.run(args.steps, args.warmup, world, pre=PRE_ROLL_CYCLES * env_s.refill_every)
            strong = {"value": rs["value"], "unit": "env-steps/s", "scaling": "strong", "n_gpus": world,
                      "num_envs_total": args.strong_envs, "num_envs_per_gpu": Es, "steps": args.steps,
                      "ms_per_step": rs["ms_per_step"], "avg_launch_us": rs["launch_s"] * 1e6,
                      "note": "BASELINE.json's num_envs=65536 split over the ranks (env_offset = rank * E / N); "
                              "same timing rule as the headline (max over ranks, refill share charged)"}
            del run_s, env_s
            torch.cuda.synchronize()

    copy_peak = measure_copy_peak(dev)

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
        dqn = dqn_consumer_bench(env, actions, rewards, dones, obs, args.warmup, min(args.steps, 200), stream,
                                 args.loop_precision, loop_input(args, env))

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
        loop = train_loop_bench(env, args.loop_segments, parallel=args.parallel_loop, fused=not args.unfused_act,
                                precision=args.loop_precision, input=loop_input(args, env))
        loop["env_steps_per_s"] = min_over_ranks(loop["env_steps_per_s"], world) * world
        loop["us_per_step"] = max_over_ranks(loop["us_per_step"], world)
        loop["n_gpus"] = world
        loop["num_envs_total"] = E * world
    del runner, actions, rewards, dones, obs, env

    # ---- the north-star configuration (BASELINE.json north_star, SURVEY.md
    # §8 D2 C5): 64x64 grid, 32 drones, c5_envs per rank (2^20 over 8 GPUs),
    # step + obs(K=1) with refills, >= 200 timed steps
    c5 = None
    if north:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        env5, G5, N5, E5, K5 = make_env("c5", args.c5_envs, rank, dev)
        st5 = env5.default_obs_stream
        steps5 = max(args.c5_steps, 200)
        run5 = StepRunner(env5, K5, steps5 + 20 + 2 * env5.refill_every, st5)
        r5 = run5.run(steps5, 20, world, pre=PRE_ROLL_CYCLES * env5.refill_every)
        R5, W5 = algorithmic_bytes(G5, N5, K5, env5.layout.obs_window)
        c5 = {"value": r5["value"], "unit": "env-steps/s", "n_gpus": world, "steps": steps5, "warmup": 20,
              "ms_per_step": r5["ms_per_step"], "wall_ms_per_step": r5["wall_ms_per_step"],
              "config": {"workload": f"C5 (north star): {G5}x{G5} grid, {N5} drones, {E5} envs/GPU, "
                                     f"step + fused obs(K={K5})", "num_envs_per_gpu": E5,
                         "num_envs_total": E5 * world, "obs_stores": "streaming" if st5 else "cached",
                         "parallelism": f"env-shard x{world}"},
              "roofline": roofline(E5, R5, W5, r5["launch_s"], r5["refill"], traffic_of("c5"), G5, copy_peak),
              "refill": r5["refill"],
              "train_loop": None,
              "north_star": "BASELINE.json: >= 1e8 env-steps/s at num_envs=2^20 on 8 GPUs at >= 40% HBM-read "
                            "roofline (roofline.frac)"}
        del run5
        # BASELINE.json configs[4]: "full scan-style train loop" at the C5 shape
        # (train_jax.py:38-115, :215-236), the same graph-captured 100-step
        # segments + reset as `train_loop`, c5_envs per rank
        if args.loop_segments > 0 and not args.no_dqn and K5 >= 1:
            l5 = train_loop_bench(env5, args.loop_segments, parallel=args.parallel_loop, fused=not args.unfused_act,
                                  precision=args.loop_precision, input=loop_input(args, env5))
            l5["env_steps_per_s"] = min_over_ranks(l5["env_steps_per_s"], world) * world
            l5["us_per_step"] = max_over_ranks(l5["us_per_step"], world)
            l5["n_gpus"] = world
            l5["num_envs_total"] = E5 * world
            c5["train_loop"] = l5
        del env5

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(G, N, K, args.cpu_seconds)

    if rank == 0:
        with open(os.path.join(REPO, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
        out = {
            "metric": metric,
            "value": main_res["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic uniform random actions (counter hash), envs seeded random.seed(env index)",
            "config": {"workload": f"{args.config.upper()}: {G}x{G} grid, {N} drones, {E} envs/GPU, "
                                   f"step + fused obs(K={K}) + the drl_refill share",
                       "grid": G, "n_drones": N, "num_envs_per_gpu": E, "num_envs_total": E * world,
                       "obs_k": K, "obs_stores": "streaming" if args.obs_stream else "cached",
                       "parallelism": f"env-shard x{world}",
                       "setup": f"reset(seed=0), then {PRE_ROLL_CYCLES * main_res['refill']['every']} pre-roll steps "
                                f"({PRE_ROLL_CYCLES} refill cycles: steady-state candidate rings) before the warm-up"},
            "wall_ms_per_step": main_res["wall_ms_per_step"],
            "roofline": roofline(E, R, Wb, main_res["launch_s"], main_res["refill"], traffic_of(args.config), G,
                                 copy_peak),
            "refill": main_res["refill"],
            "strong": strong,
            ("cached_obs" if args.obs_stream else "streaming_obs"): other,
            "c5": c5,
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
