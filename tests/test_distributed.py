"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path.

The env step itself needs a GPU, so the episode runner here is backed by the
oracle (tests may use it as the checker); what is exercised is the product's
sharding arithmetic, seeding by global env index, and the eval all-reduce.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dronerl_amd.distributed import evaluate_sharded, shard_envs, shard_episodes


def test_shard_envs_rules():
    s = [shard_envs(65536 * 8, r, 8) for r in range(8)]
    assert [x.env_offset for x in s] == [65536 * r for r in range(8)]
    assert all(x.num_envs == 65536 for x in s)
    with pytest.raises(ValueError, match="divisible"):
        shard_envs(10, 0, 4)
    with pytest.raises(ValueError):
        shard_envs(0, 0, 1)
    eps = [shard_episodes(10, r, 4) for r in range(4)]
    assert sum(len(e) for e in eps) == 10 and eps[0].start == 0 and eps[-1].stop == 10


def oracle_runner(n_drones=3, side=8, steps=50, eval_seed=100):
    def run(eps):
        from oracle.oracle import OracleMulti, Params, synth_actions
        o = OracleMulti(Params(side=side, n_drones=n_drones), len(eps))
        o.reset(eval_seed + np.arange(eps.start, eps.stop))
        sums = np.zeros((len(eps), 2))
        for t in range(steps):
            a = synth_actions(0, t, np.arange(eps.start, eps.stop), n_drones)
            r, _ = o.step(a)
            sums[:, 0] += r[:, 0]
            sums[:, 1] += r[:, 1]
        return torch.from_numpy(sums / steps)
    return run


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        agent, rnd, table = evaluate_sharded(oracle_runner(), num_evals=7, rank=rank, world=world)
        # max-over-ranks timing reduction used by bench.py
        from dronerl_amd.distributed import max_over_ranks
        m = max_over_ranks(float(rank + 1))
        out[rank] = (agent, rnd, table.numpy().tolist(), m)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_eval_allreduce_two_ranks_matches_single_process():
    ref_agent, ref_rnd, ref_table = evaluate_sharded(oracle_runner(), num_evals=7)
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
            assert p.exitcode == 0
        res = dict(out)
    for r in range(2):
        agent, rnd, table, m = res[r]
        np.testing.assert_allclose(np.array(table), ref_table.numpy(), rtol=0, atol=0)
        assert agent == pytest.approx(ref_agent) and rnd == pytest.approx(ref_rnd)
        assert m == 2.0
