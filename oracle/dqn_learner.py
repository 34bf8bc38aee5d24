"""ORACLE — TEST INFRASTRUCTURE ONLY (not part of the product).

numpy restatement of one DQN learner step, the checker of drl_dqn_train
(dronerl_amd/csrc/dronerl_learn.hip).  Only ``tests/`` may import it.

What it restates (reference file:line):
  * train_jax.py:68-98 -- per scan step: ``train_if_can_sample`` when
    ``buffer.can_sample`` (jax_impl/buffers.py:92-93: size >= batch), then
    ``update_target`` when ``step % target_update_interval == 0``, then
    ``update_epsilon`` when ``step % epsilon_decay_every == 0``; step + 1.
  * jax_impl/buffers.py:79-90 ``sample`` -- uniform rows in [0, size) (rows drawn
    by the build's counter hash, ``sample_indices``; the reference's
    jax.random.randint stream is jax-only: parity unpinned for the draw).
  * jax_impl/agents/dqn.py:147-183 ``train_step`` -- q = Q(obs)[action],
    td = reward + gamma * max_a Q_target(next_obs) * (1 - done),
    loss = mean((q - td)^2), jax.value_and_grad, optax.adam update;
    dqn.py:47-57 DenseQNetwork (Dense + relu per hidden layer, Dense(5)).
  * dqn.py:185-190 ``update_target`` -- optax.incremental_update:
    tau * new + (1 - tau) * old.
  * dqn.py:192-200 ``update_epsilon`` -- max(epsilon * decay, end).
  * optax.adam (optax 0.2.x scale_by_adam + scale(-lr); not importable here,
    its published formula restated): mu = (1 - b1) g + b1 mu,
    nu = (1 - b2) g^2 + b2 nu, u = (mu / (1 - b1^t)) / (sqrt(nu / (1 - b2^t))
    + eps), p + u * (-lr).

Arithmetic is float32 with every product and sum rounded in the kernel's
order (the kernel compiles with contraction off): a dot product keeps four
partial sums over k mod 4, each accumulated in k order, combined
(s0 + s1) + (s2 + s3), then + bias; sums over the batch run row by row from
0.0.  The constants are what jax's weak typing makes of python floats
(``1 - b1`` computed in double, then rounded to f32); b^t is a running double
product rounded once per use.  tests/test_dqn_learner.py pins this
restatement against torch autograd + the written-out optax formula.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

F = np.float32
M64 = (1 << 64) - 1
OBJ_SKYSCRAPER, OBJ_STATION, OBJ_DROPZONE, OBJ_PACKET = 2, 3, 4, 5  # common/constants.py Object


def _mix(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sample_indices(seed: int, step: int, batch: int, size: int) -> List[int]:
    """The learner's rows for scan step `step` (dronerl_learn.hip dq_sample)."""
    out = []
    for b in range(batch):
        h = _mix((seed & M64) ^ _mix(((step & 0xFFFFFFFF) << 16) | b))
        out.append(((h >> 32) * size) >> 32)
    return out


def decode_code_rows(rows: np.ndarray, W: int) -> np.ndarray:
    """Policy-code rows uint8 [n, code_bytes] -> f32 [n, W*W*6] with the
    channel rules of torch_impl/env/wrappers.py:10-31 (as drl_code_decode)."""
    n = rows.shape[0]
    cells = W * W
    cpg = -(-cells // 4)
    cpg8 = -(-cpg // 8) * 8
    c = np.ascontiguousarray(rows).view(np.uint16).reshape(n, 4, cpg8)
    h = np.zeros((n, cells), np.uint32)
    for g in range(4):
        k = min(cpg, cells - g * cpg)
        if k > 0:
            h[:, g * cpg:g * cpg + k] = c[:, g, :k]
    obj, air = h & 7, h >> 3
    out = np.zeros((n, cells, 6), F)
    out[..., 0] = air != 0
    out[..., 1] = (obj == OBJ_PACKET) | ((air & 0x80) != 0)
    out[..., 2] = obj == OBJ_DROPZONE
    out[..., 3] = obj == OBJ_STATION
    charge = ((air & 0x7F).astype(np.int64) - 1).astype(F) / F(100.0)
    out[..., 4] = np.where(air != 0, charge, F(0.0))
    out[..., 5] = obj == OBJ_SKYSCRAPER
    return out.reshape(n, cells * 6)


def dot4(X: np.ndarray, Wt: np.ndarray) -> np.ndarray:
    """X [B, n] . W[out, n]^T with the learner's summation order -> [B, out]."""
    B, n = X.shape
    s = np.zeros((4, B, Wt.shape[0]), F)
    for k in range(n):
        s[k & 3] = s[k & 3] + X[:, k, None] * Wt[None, :, k]
    return (s[0] + s[1]) + (s[2] + s[3])


def backprop4(D: np.ndarray, Wt: np.ndarray) -> np.ndarray:
    """D [B, out] . W [out, in] with the same order over the out index -> [B, in]."""
    B, out = D.shape
    s = np.zeros((4, B, Wt.shape[1]), F)
    for j in range(out):
        s[j & 3] = s[j & 3] + D[:, j, None] * Wt[None, j, :]
    return (s[0] + s[1]) + (s[2] + s[3])


@dataclass
class HParams:
    """train_jax.py's learner arguments (defaults :349-360; optax.adam's)."""
    batch: int = 8
    gamma: float = 0.9
    learning_rate: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-8
    tau: float = 1.0
    target_update_interval: int = 10
    epsilon_decay: float = 0.999
    epsilon_end: float = 0.01
    epsilon_decay_every: int = 5
    sample_seed: int = 0


@dataclass
class LearnerState:
    """Parameter sets as lists of (W [out][in], b [out]) float32 arrays."""
    online: list
    target: list
    m: list
    v: list
    step: int = 0
    count: int = 0
    epsilon: np.float32 = field(default_factory=lambda: F(1.0))
    loss: np.float32 = field(default_factory=lambda: F(0.0))
    beta1_pow: float = 1.0
    beta2_pow: float = 1.0

    @staticmethod
    def start(online, target, epsilon_start: float) -> "LearnerState":
        z = [(np.zeros_like(w), np.zeros_like(b)) for w, b in online]
        return LearnerState([(w.astype(F).copy(), b.astype(F).copy()) for w, b in online],
                            [(w.astype(F).copy(), b.astype(F).copy()) for w, b in target],
                            copy.deepcopy(z), copy.deepcopy(z), epsilon=F(epsilon_start))


def forward(params, X: np.ndarray):
    """DenseQNetwork (dqn.py:50-57): returns (pre-activations per layer,
    activations per hidden layer, q)."""
    zs, hs = [], []
    a = X
    for i, (w, b) in enumerate(params):
        z = dot4(a, w) + b[None, :]
        zs.append(z)
        if i < len(params) - 1:
            a = np.where(z > 0, z, F(0.0)).astype(F)
            hs.append(a)
    return zs, hs, zs[-1]


def _adam(hp: HParams, p, g, m, v, bc1, bc2):
    c1, c2 = F(1.0 - hp.beta1), F(1.0 - hp.beta2)
    m2 = c1 * g + F(hp.beta1) * m
    v2 = c2 * (g * g) + F(hp.beta2) * v
    u = (m2 / bc1) / (np.sqrt(v2 / bc2) + F(hp.adam_eps))
    return (p + u * F(-hp.learning_rate)).astype(F), m2.astype(F), v2.astype(F)


def learner_step(st: LearnerState, hp: HParams, obs: np.ndarray, next_obs: np.ndarray, actions: np.ndarray,
                 rewards: np.ndarray, dones: np.ndarray, size: int, code_window: int = 0) -> dict:
    """One learner block of a train_jax.py scan step on a replay whose rows
    are `obs` / `next_obs` (f32 [capacity, >= in] or policy-code uint8 rows
    with code_window = W), actions i32, rewards f32, dones u8 [capacity];
    `size` = current_size.  Updates `st` in place; returns the step's rows
    and the loss."""
    step = st.step
    info = {"trained": size >= hp.batch, "rows": None, "loss": F(0.0)}
    if size >= hp.batch:
        idx = sample_indices(hp.sample_seed, step, hp.batch, size)
        info["rows"] = idx
        n_in = st.online[0][0].shape[1]
        if code_window:
            X = decode_code_rows(obs[idx], code_window)
            Xn = decode_code_rows(next_obs[idx], code_window)
        else:
            X = obs[idx, :n_in].astype(F)
            Xn = next_obs[idx, :n_in].astype(F)
        zs, hs, q = forward(st.online, X)
        _, _, qt = forward(st.target, Xn)
        B = hp.batch
        A = q.shape[1]
        d = np.zeros(B, F)
        act = np.zeros(B, np.int64)
        for b in range(B):
            s = idx[b]
            mx = qt[b, 0]
            for j in range(1, A):
                mx = qt[b, j] if qt[b, j] > mx else mx
            notdone = F(0.0) if dones[s] else F(1.0)
            td = F(rewards[s]) + (F(hp.gamma) * mx) * notdone
            a = int(actions[s])
            ok = 0 <= a < A
            d[b] = (q[b, a] if ok else td) - td
            act[b] = a if ok else -1
        loss = F(0.0)
        for b in range(B):
            loss = F(loss + d[b] * d[b])
        loss = F(loss / F(B))
        D = np.zeros((B, A), F)
        for b in range(B):
            if act[b] >= 0:
                D[b, act[b]] = (d[b] + d[b]) / F(B)
        st.beta1_pow *= hp.beta1
        st.beta2_pow *= hp.beta2
        bc1, bc2 = F(1.0 - st.beta1_pow), F(1.0 - st.beta2_pow)
        L = len(st.online)
        deltas = [None] * L
        deltas[L - 1] = D
        for l in range(L - 1, 0, -1):
            dh = backprop4(deltas[l], st.online[l][0])
            deltas[l - 1] = np.where(hs[l - 1] > 0, dh, F(0.0)).astype(F)
        inputs = [X] + hs
        new_online, new_m, new_v = [], [], []
        for l in range(L):
            w, b = st.online[l]
            mw, mb = st.m[l]
            vw, vb = st.v[l]
            Dl = deltas[l]
            gw = np.zeros_like(w)
            gb = np.zeros_like(b)
            for r in range(B):
                gw = gw + Dl[r][:, None] * inputs[l][r][None, :]
                gb = gb + Dl[r]
            w2, mw2, vw2 = _adam(hp, w, gw, mw, vw, bc1, bc2)
            b2, mb2, vb2 = _adam(hp, b, gb, mb, vb, bc1, bc2)
            new_online.append((w2, b2))
            new_m.append((mw2, mb2))
            new_v.append((vw2, vb2))
        st.online, st.m, st.v = new_online, new_m, new_v
        st.count += 1
        info["loss"] = loss
        info["deltas"] = deltas
        info["grads_inputs"] = inputs
    st.loss = info["loss"]
    if step % hp.target_update_interval == 0:
        tau, omt = F(hp.tau), F(1.0 - hp.tau)
        st.target = [((tau * w + omt * tw).astype(F), (tau * b + omt * tb).astype(F))
                     for (w, b), (tw, tb) in zip(st.online, st.target)]
    if step % hp.epsilon_decay_every == 0:
        e = F(st.epsilon * F(hp.epsilon_decay))
        st.epsilon = e if e > F(hp.epsilon_end) else F(hp.epsilon_end)
    st.step = step + 1
    return info


def train_jax_epsilon_decay(num_steps: int, epsilon_start: float = 1.0, epsilon_end: float = 0.01,
                            half_life_fraction: float = 0.2) -> float:
    """train_jax.py:133-134: the decay that halves epsilon's distance to the
    end value after half_life_fraction of the run (per decay call)."""
    return (1 - 0.5 * (1 - epsilon_end / epsilon_start)) ** (1 / (half_life_fraction * num_steps))


def run(st: LearnerState, hp: HParams, replay: dict, sizes, code_window: int = 0) -> list:
    """Several learner steps (one per entry of `sizes`); returns the infos."""
    return [learner_step(st, hp, replay["obs"], replay["next_obs"], replay["actions"], replay["rewards"],
                         replay["dones"], s, code_window) for s in sizes]


def flat(params) -> Optional[np.ndarray]:
    """Concatenated W, b of each layer (torch state_dict order)."""
    return np.concatenate([np.concatenate([w.ravel(), b.ravel()]) for w, b in params])
