"""CPU checks of bench.py's measurement pieces (no GPU): the survey's
algorithmic bytes per env-step, the committed PMC traffic
bench.py reports, the CPU-baseline record and the command-line contract."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("cfg,R,W", [("c2", 296, 1504), ("c3", 296, 1504), ("c4", 1104, 2344),
                                     ("c5", 4256, 5560)])
def test_algorithmic_bytes_match_survey_d3(cfg, R, W):
    G, N, _, K = bench.CONFIGS[cfg]
    assert bench.algorithmic_bytes(G, N, K) == (R, W)


def test_headline_config_is_c3():
    assert bench.CONFIGS["c3"] == (16, 8, 65536, 1)
    assert bench.CONFIGS["c5"][2] * 8 == 2 ** 20  # north star: 2^20 envs over 8 GPUs


@pytest.mark.parametrize("cfg", ["c3", "c4", "c5"])
def test_committed_traffic_is_read_plus_doubled_fetch(cfg):
    path = os.path.join(REPO, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        pytest.skip(f"no {path}")
    with open(path) as f:
        d = json.load(f)
    pmc = d["pmc_mean_per_launch"]
    # MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE counts half the bytes (KiB units)
    expect = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
    assert abs(d["hbm_bytes_per_launch"] - expect) <= 1e-6 * expect
    assert bench.load_traffic(cfg) == d["hbm_bytes_per_launch"]
    G, N, E, K = bench.CONFIGS[cfg]
    R, W = bench.algorithmic_bytes(G, N, K)
    # measured traffic per env-step within a factor of 2 of the algorithmic bytes; the lower bound takes the
    # ground as packed (ABI 8: G^2 / 2 bytes read) and not written back whole (only changed cells are)
    per = d["hbm_bytes_per_launch"] / E
    assert 0.5 * (R - G * G // 2 + W - G * G) < per < 2.0 * (R + W)


def test_cpu_baseline_record():
    rec = bench.cpu_baseline(8, 4, 1, seconds=0.4)
    assert rec["kind"] == "port" and rec["unit"] == "env-steps/s"
    assert rec["value"] > 0 and rec["single_thread_value"] > 0
    assert rec["cores"] == bench.host_cpus()[0] <= len(os.sched_getaffinity(0))  # the lease's CPUs (§8 D4)
    assert "affinity" in rec["cores_basis"]
    assert "envs x" in rec["sample"]


def test_cli_help_lists_contract_flags():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True,
                         text=True, timeout=120, check=True).stdout
    for flag in ("--gpus", "--steps", "--warmup", "--config", "--cached-steps", "--no-pmc-traffic", "--c5-envs",
                 "--loop-precision"):
        assert flag in out


def test_no_nested_profiler_inside_a_rocprofv3_run(monkeypatch):
    """Inside a rocprofv3 run the GPU is already initialised by its tool, so
    bench.py must not start its own rocprofv3 children (they exec their
    target): the in-run traffic passes are skipped."""
    for k in [k for k in os.environ if k.startswith("ROCPROF")]:
        monkeypatch.delenv(k)
    monkeypatch.setenv("LD_PRELOAD", "")
    assert not bench.under_profiler()
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert bench.under_profiler()
    monkeypatch.delenv("ROCPROF_OUTPUT_PATH")
    monkeypatch.setenv("LD_PRELOAD", "/opt/rocm/lib/librocprofiler-sdk-tool.so")
    assert bench.under_profiler()
    assert bench.measure_traffic(None, ["c3"]) is None  # returns before reading any argument


@pytest.mark.parametrize("pre,warmup,steps,every", [(32, 5, 20, 32), (32, 50, 1000, 32), (32, 50, 200, 32),
                                                    (25, 5, 20, 25), (32, 0, 64, 32), (1, 0, 7, 1)])
def test_refill_share_charged_at_any_step_count(pre, warmup, steps, every):
    """the timed region carries exactly steps/every refills
    (the ones inside it plus a prorated share), so the driver's 20-step run
    is charged like a 1000-step one."""
    inside, charge = bench.refill_plan(pre, warmup, steps, every)
    first = pre + warmup
    assert inside == [s for s in range(first, first + steps) if (s + 1) % every == 0]
    assert len(inside) + charge == pytest.approx(steps / every)
    assert -1.0 < charge < 1.0
    if not inside:
        assert charge > 0  # e.g. --steps 20 --warmup 5: no refill inside, 0.625 of one charged


def test_driver_run_charges_a_refill():
    inside, charge = bench.refill_plan(bench.PRE_ROLL_CYCLES * 32, 5, 20, 32)
    assert inside == [] and charge == pytest.approx(20 / 32)


def test_pre_roll_prices_the_refill_in_steady_state():
    """The pro-rated refill of a short run is priced by the pre-roll's refills
    minus the first two after the reset (lighter than the steady state):
    enough cycles remain to average."""
    assert bench.PRE_ROLL_CYCLES - 2 >= 4


def test_roofline_fractions_stay_below_one():
    """every reported fraction is a share of the HBM peak
    that the kernel can reach: R-only, measured traffic / time (no read+write
    figure whose W counts a ground write-back the kernel never does)."""
    E, R, Wb = 131072, 4256, 5560
    refill = {"every": 32, "per_step_us": 5.0}
    traffic = {"drl_step_kernel": {"bytes_per_launch": 810e6, "read_bytes_per_launch": 600e6,
                                   "write_bytes_per_launch": 210e6},
               "drl_refill_kernel": {"bytes_per_launch": 400e6, "read_bytes_per_env": 2000.0,
                                     "write_bytes_per_env": 1000.0}, "source": "test", "envs": E}
    rl = bench.roofline(E, R, Wb, 143.6e-6, refill, traffic)

    def fracs(d):
        for k, v in d.items():
            if isinstance(v, dict):
                yield from fracs(v)
            elif k.startswith("frac"):
                yield k, v
    found = dict(fracs(rl))
    assert "frac_read_plus_write" not in found and "frac_measured" in found
    assert all(0.0 < v <= 1.0 for v in found.values()), found


@pytest.mark.parametrize("kern", ["drl_refill_list_kernel", "drl_refill_kernel"])
def test_refill_traffic_from_either_refill_form(kern):
    """The refill's PMC bytes enter `with_refill` whichever form ran: the
    worklist kernel (the default since round 3) or the wave-per-env kernel
    (DRL_REFILL_LIST=0); the child's grid sizes tell their rows apart."""
    E, R, Wb = 65536, 296, 1504
    refill = {"every": 32, "per_step_us": 1.45}
    traffic = {"drl_step_kernel": {"bytes_per_launch": 118e6, "read_bytes_per_launch": 35e6,
                                   "write_bytes_per_launch": 83e6},
               kern: {"bytes_per_launch": 180e6, "read_bytes_per_env": 1267.0, "write_bytes_per_env": 1481.0},
               "source": "test", "envs": E}
    wr = bench.roofline(E, R, Wb, 20.0e-6, refill, traffic)["with_refill"]
    assert wr["refill_traffic_per_launch"] == 180e6
    assert wr["traffic_per_step"] == pytest.approx(118e6 + 180e6 / 32)
    assert set(bench.PMC_KERNELS) >= {"drl_step_kernel", "drl_refill_list_kernel", "drl_refill_kernel"}


@pytest.mark.parametrize("cfg,launch_us", [("c3", 19.83), ("c3", 14.0), ("c4", 28.0), ("c5", 143.6), ("c5", 110.0),
                                            ("c5", 70.0)])
def test_no_ceiling_below_its_frac(cfg, launch_us):
    """VERDICT r3 item 8 / ADVICE r4: every `*ceiling*` field bounds its frac.
    frac_ceiling = R / ((R - G^2/2) + (W - G^2)): the obligatory bytes are
    the ground as stored (two cells per byte) and the outputs; a launch that
    moves them at or below the spec peak takes at least t_min, and then frac
    <= frac_ceiling (at C5 the ceiling exceeds 1: R counts G^2 ground bytes,
    the kernel reads G^2/2)."""
    G, N, E, K = bench.CONFIGS[cfg]
    R, Wb = bench.algorithmic_bytes(G, N, K)
    refill = {"every": 32, "per_step_us": 2.0}
    peak = {"copy_GBs": 6290.0, "read_GBs": 5900.0, "note": "test"}
    rl = bench.roofline(E, R, Wb, launch_us * 1e-6, refill, None, G, peak)
    obligatory = (R - G * G // 2) + (Wb - G * G)
    assert rl["frac_ceiling"] == pytest.approx(R / obligatory)
    t_min = E * obligatory / (bench.PEAK_HBM_GBS * 1e9)
    if launch_us * 1e-6 >= t_min:
        assert rl["frac"] <= rl["frac_ceiling"]
        ceilings = {k: v for k, v in rl.items() if "ceiling" in k}
        assert ceilings and all(v >= rl["frac"] for v in ceilings.values())
    assert rl["frac_vs_measured_peak"] == pytest.approx(rl["achieved"] / 6290.0)


@pytest.mark.parametrize("probe,kernel_GBs", [(6290.0, 5760.0), (4800.0, 5760.0), (6300.0, None)])
def test_measured_peak_fractions_at_most_one(probe, kernel_GBs):
    """the measured peak is a peak -- the best of the
    probe's copy / read rates and the kernel's own measured traffic rate -- so
    every *_vs_measured_peak field is <= 1 (round 4's 4.80 TB/s probe gave
    1.21 against a 5.76 TB/s step)."""
    E, R, Wb, G = 65536, 296, 1504, 16
    launch_s = 19.0e-6
    traffic = None
    if kernel_GBs:
        b = kernel_GBs * 1e9 * launch_s
        traffic = {"drl_step_kernel": {"bytes_per_launch": b, "read_bytes_per_launch": 0.3 * b,
                                       "write_bytes_per_launch": 0.7 * b}, "source": "test", "envs": E}
    peak = {"copy_GBs": probe, "read_GBs": probe * 0.95, "note": "test"}
    rl = bench.roofline(E, R, Wb, launch_s, {"every": 32, "per_step_us": 1.2}, traffic, G, peak)
    vs = {k: v for k, v in rl.items() if k.endswith("vs_measured_peak")}
    assert vs and all(0.0 < v <= 1.0 for v in vs.values()), vs
    assert rl["peak_measured"] == max(probe, kernel_GBs or 0.0)
    assert rl["peak_measured_source"] == ("drl_hbm_probe copy" if probe >= (kernel_GBs or 0) else
                                          "drl_step_kernel traffic")


def test_visible_gpus_counts_without_hip(monkeypatch):
    """the launcher counts GPUs from the KFD topology (no HIP call),
    narrowed by the *_VISIBLE_DEVICES variables."""
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: (_ for _ in ()).throw(AssertionError("HIP")))
    n = bench.visible_gpus()
    assert n is None or n >= 0
    if n:
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
        assert bench.visible_gpus() == 1


def test_act_code_flops_count():
    """the code act's MFMA count per 16-env tile (layer 0:
    10 K-slices x 8 unit tiles x 2; layer 1: 4 x 4 x 3; output: 2 x 1 x 3)."""
    ex, alg, per_tile = bench.act_code_flops(65536, 7)
    assert per_tile == 10 * 8 * 2 + 4 * 4 * 3 + 2 * 1 * 3 == 214
    assert ex == 4096 * 214 * 2 * 16 * 16 * 32
    assert alg == 2 * 65536 * (294 * 128 + 128 * 64 + 64 * 5)
    rl = bench.act_code_roofline(65536, 7, 21.75e-6)
    assert rl["bound"] == "mfma" and rl["unit"] == "TFLOP/s"
    assert rl["frac"] == pytest.approx(ex / 21.75e-6 / 1e12 / bench.MFMA_PEAK_TFLOPS)


def test_launcher_plumbing(monkeypatch):
    """`bench.py --gpus N` with no torch.distributed.run
    environment starts its own N ranks as a child job (never an exec, before
    any GPU call) with the same arguments; under torchrun (WORLD_SIZE set),
    or for one GPU, or in a PMC child, it runs in-process."""
    import argparse
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    ns = lambda gpus, pmc="": argparse.Namespace(gpus=gpus, pmc_child=pmc)  # noqa: E731
    assert bench.needs_launch(ns(8)) and bench.needs_launch(ns(2))
    assert not bench.needs_launch(ns(1)) and not bench.needs_launch(ns(8, "c3"))
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert not bench.needs_launch(ns(8))
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.launcher_command(argv, 8, 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29517" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(REPO, "bench.py") and cmd[-len(argv):] == argv
    assert 1024 <= bench.free_port() < 65536


def test_launcher_refuses_more_nccl_ranks_than_gpus(monkeypatch, capsys):
    """No GPU here: nccl (RCCL) needs one device per rank, so the launcher
    refuses before starting anything (exit 2); gloo may share devices."""
    monkeypatch.setattr(bench, "DIST_BACKEND", "nccl")
    monkeypatch.setattr(bench, "visible_gpus", lambda: 0)
    assert bench.launch_ranks(["--gpus", "2"], 2) == 2
    assert "one GPU per rank" in capsys.readouterr().err


def test_strong_split():
    """BASELINE.json's num_envs=65536 over 1/2/4/8 ranks."""
    assert [bench.strong_split(65536, n) for n in (1, 2, 4, 8)] == [65536, 32768, 16384, 8192]
    with pytest.raises(ValueError, match="divisible"):
        bench.strong_split(65536, 3)
    with pytest.raises(ValueError):
        bench.strong_split(0, 2)


def test_cpu_baseline_quotes_reference_torch_impl():
    """the reference's own torch_impl step()+WindowedGridView,
    timed in the build container by oracle/time_reference_torch_impl.py, is
    quoted beside the port baseline and labelled as other hardware."""
    import bench
    for G, N in ((16, 8), (64, 32)):
        r = bench.reference_torch_impl(G, N)
        assert r is not None and r["kind"] == "reference" and r["different_hardware"] is True
        assert r["value"] > 0 and r["step_only_value"] > r["value"] and r["cores"] == 1
        assert "NOT the GPU box" in r["hardware"]
    assert bench.reference_torch_impl(12, 3) is None
