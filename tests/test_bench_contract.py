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
    # measured traffic per env-step within a factor of 2 of the algorithmic bytes
    per = d["hbm_bytes_per_launch"] / E
    assert 0.5 * (R + W) < per < 2.0 * (R + W)


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
