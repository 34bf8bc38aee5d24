#!/usr/bin/env python3
"""Diagnostic: time drl_qnet_act alone (HIP events) for a library variant."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--hidden", default="128,64")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--stride", type=int, default=294, help="obs row stride in floats (296: 16-B aligned rows)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--input", default="obs", choices=["obs", "code"], help="code: drl_qnet_act_code (f32)")
    ap.add_argument("--synth", action="store_true", help="also write drones 1..N-1's synthetic actions (act_synth)")
    ap.add_argument("--drones", type=int, default=8, help="action columns (N; the train loop's act writes N - 1 "
                    "synthetic ones with --synth: 31 at C5)")
    ap.add_argument("--stamps", action="store_true", help="library built with -DDRL_QC_STAMPS: phase cycles")
    ap.add_argument("--slices", type=int, default=0, help="v4 stamps: layer-0 slices per pass to print (10 at 7x7)")
    ap.add_argument("--group", type=int, default=64,
                    help="envs per wave pass of the stamped code act (64: v4 kernel, 32: DRL_QN_CODE=2|3)")
    ap.add_argument("--flush", action="store_true",
                    help="overwrite 256 MB between launches (cold L2/MALL, as after a step) and time each launch")
    ap.add_argument("--rewrite", action="store_true", help="with --flush: rewrite the input rows after the flush "
                    "(freshly written, as the step leaves its codes)")
    ap.add_argument("--repack", action="store_true", help="with --flush: re-pack the net after the flush "
                    "(a freshly written packed image, as the learner leaves it)")
    ap.add_argument("--retouch", action="store_true", help="with --flush: rewrite the packed image with a torch "
                    "copy (the same bytes, whole-line stores)")
    args = ap.parse_args()
    if args.lib:
        import dronerl_amd._native as nat
        nat.LIB_PATH = os.environ["DRL_LIB"] = os.path.abspath(args.lib)
    from dronerl_amd.dqn import QNetwork
    E = args.envs
    obs = torch.rand((E, 1, 7, 7, 6), device="cuda")
    net = QNetwork(294, tuple(int(x) for x in args.hidden.split(",")), generator=torch.Generator().manual_seed(0),
                   precision=args.precision, input=args.input)
    a = torch.zeros((E, args.drones), dtype=torch.int32, device="cuda")
    flat = obs.reshape(E, -1)
    if args.stride != 294:
        big = torch.zeros((E, args.stride), device="cuda")
        big[:, :294] = flat
        flat = big[:, :294]
    if args.input == "code":  # real codes from a C3 env (drone 0's window)
        from dronerl_amd import BatchedDeliveryDrones, EnvParams
        env = BatchedDeliveryDrones(EnvParams(n_drones=8, grid_size=16), E)
        env.reset(seed=0)
        flat = env.new_code()
        for t in range(4):
            env.step(env.synth_actions(seed=1, step=t), obs_k=1, code=flat)
    for _ in range(20):
        net.act(flat, 0.1, actions=a)
    syn = (lambda t: (5, t)) if args.synth else (lambda t: None)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if args.flush:
        junk = torch.empty(64 << 20, dtype=torch.float32, device="cuda")
        tot = 0.0
        keep = flat.clone() if args.rewrite else None
        for t in range(args.iters):
            junk.fill_(float(t))
            if args.rewrite:
                flat.copy_(keep)
            if args.repack:
                net.pack()
            if args.retouch:
                net.packed.copy_(net.packed.clone())
            e0.record()
            net.act(flat, 0.1, step=t, actions=a, synth=syn(t))
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        us = tot * 1e3 / args.iters
    else:
        e0.record()
        for t in range(args.iters):
            net.act(flat, 0.1, step=t, actions=a, synth=syn(t))
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
    if args.stamps:
        q = torch.zeros((E, 5), device="cuda")
        net.act(flat, 0.1, actions=a, q_out=q)
        torch.cuda.synchronize()
        gr = args.group if args.input == "code" and args.hidden in ("128,64", "128,32") else 16
        rows = (E + gr - 1) // gr
        st = q.view(torch.int32).cpu().numpy().astype("int64").reshape(-1)[: 5 * rows].reshape(rows, 5)
        import numpy as np
        for i, name in enumerate(("layer0", "hidden" if rows == (E + 15) // 16 else "layer1",
                                  "epilogue" if rows == (E + 15) // 16 else "layer2+epilogue")):
            v = st[:, i]
            print(f"stamps {name}: median {np.median(v):.0f} p10 {np.percentile(v, 10):.0f} "
                  f"p90 {np.percentile(v, 90):.0f} cycles (s_memtime)")
        nw = min(rows, 1024)  # the first pass of every wave (256 CUs x 4 waves) vs later passes
        if rows > nw:
            for lab, sel in (("first pass", st[:nw]), ("later passes", st[nw:])):
                print(f"  {lab}: " + " ".join(f"{n} {np.median(sel[:, i]):.0f}" for i, n in
                                              enumerate(("layer0", "layer1", "layer2+epi"))))
        if args.slices:  # v4 stamps build: per-slice layer-0 times after the 5-word rows
            allw = q.view(torch.int32).cpu().numpy().astype("int64").reshape(-1)
            sl = allw[5 * rows: 5 * rows + args.slices * rows].reshape(rows, args.slices)
            print("layer-0 slice ends (median cycles since the pass start): " +
                  " ".join(f"{np.median(sl[:, i]):.0f}" for i in range(args.slices)))
        t0 = st[:, 3] & 0xffffffff
        t3 = st[:, 4] & 0xffffffff
        print(f"tile start since kernel entry: min {t0.min()} median {np.median(t0):.0f} max {t0.max()}; "
              f"tile end: median {np.median(t3):.0f} max {t3.max()} cycles")
    nb = flat.shape[1] * flat.element_size()
    print(f"{os.path.basename(args.lib) or 'libdronerl.so'} E={E} hidden={args.hidden} {args.precision} "
          f"input={args.input}{' synth' if args.synth else ''}{' flushed' if args.flush else ''}: {us:.2f} us/launch, {E * nb / us / 1e3:.0f} GB/s input read ({nb} B/env)")


if __name__ == "__main__":
    main()
