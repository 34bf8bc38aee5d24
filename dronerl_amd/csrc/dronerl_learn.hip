// dronerl_learn.hip — the DQN learner on the device (the
// train half of the consumer): one call = one train_jax.py:68-98 block of the
// scan body,
//   * buffer.can_sample -> buffer.sample -> DQNAgent.train_step
//     (jax_impl/buffers.py:79-93; jax_impl/agents/dqn.py:147-183): Q(obs)
//     gathered at the actions, target-net max over next_obs, td = r + gamma *
//     max * (1 - done), MSE, value_and_grad, optax.adam update;
//   * update_target every target_update_interval steps (dqn.py:185-190,
//     optax.incremental_update with tau);
//   * update_epsilon every epsilon_decay_every steps (dqn.py:192-200);
//   * step + 1 (the scan carry).
// Every counter (step, Adam count, epsilon, bias-correction powers) lives in
// device memory (DqnCounters), so a captured HIP graph of the loop replays a
// continuing schedule.
//
// Two launches:
//   drl_dqn_grad_kernel: the workgroups split layer 0 of both nets (online on
//     the sampled obs, target on next_obs) in 16-unit tiles; the last one to
//     arrive (agent-scope release / acquire around a ticket counter) runs the
//     later layers of both nets, the TD error, the loss, the backward pass to
//     layer 0's deltas, and the bias updates; it writes the step's plan.
//   drl_dqn_update_kernel: one thread per element of the act kernels' packed
//     net (qnet_pack_slot: each weight has exactly one): the weight's gradient
//     (sum over the batch of delta x input), the Adam update, the packed
//     fp16 hi/lo (or bf16) image the next act reads, and the target blend.
//
// Arithmetic order is fixed and contraction-free (each product rounded, then
// each sum), so oracle/dqn_learner.py reproduces the result bit for bit:
// a dot product of length n keeps four partial sums over k mod 4, each in k
// order, combined (s0 + s1) + (s2 + s3), then + bias; a batch sum runs over
// rows in order; Adam is optax's formula term by term.  The f32 constants are
// what jax's weak typing makes of the python floats (1 - b1 rounded once).
// The learner is latency-bound (a batch of 8 rows): VALU, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronerl_internal.h"

// every product and sum of this file rounds on its own (no FMA contraction): the order oracle/dqn_learner.py restates
#pragma clang fp contract(off)

namespace drl {

namespace {

__device__ __forceinline__ uint64_t dq_mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// buffers.py:79-90: B uniform indices in [0, current_size) (the reference draws
// them with jax.random.randint; here a counter hash of (seed, step, row)).
__device__ __forceinline__ int64_t dq_sample(uint64_t seed, int32_t step, int b, int64_t size) {
    const uint64_t h = dq_mix(seed ^ dq_mix(((uint64_t)(uint32_t)step << 16) | (uint64_t)b));
    return (int64_t)(((h >> 32) * (uint64_t)size) >> 32);
}

// Input k of replay row s: a policy-code row is decoded with the channel rules
// of the observation writer (wrappers.py:10-31; drl_code_decode), an f32 row read.
__device__ __forceinline__ float dq_input(const LearnArgs& a, const uint32_t* __restrict__ rows, int64_t s, int k) {
    const uint32_t* row = rows + s * a.row_words;
    if (a.code_w == 0) return __uint_as_float(row[k]);
    const int cpg = lay::code_cpg(a.code_w), cpg8 = lay::code_cpg8(a.code_w);
    const int cl = k / 6, ch = k - 6 * cl, grp = cl / cpg;
    const uint32_t h = reinterpret_cast<const uint16_t*>(row)[grp * cpg8 + (cl - grp * cpg)];
    const uint32_t obj = h & 7u, air = h >> 3;
    switch (ch) {
        case 0: return air ? 1.0f : 0.0f;
        case 1: return (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f;
        case 2: return obj == OBJ_DROPZONE ? 1.0f : 0.0f;
        case 3: return obj == OBJ_STATION ? 1.0f : 0.0f;
        case 4: return air ? (float)((int)(air & 0x7fu) - 1) / 100.0f : 0.0f;
        default: return obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f;
    }
}

// The learner's dot product (see the header): n4 float4s of x and w.
__device__ __forceinline__ float dq_dot(const float* __restrict__ x, const float* __restrict__ w, int n4) {
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    const float4* xv = reinterpret_cast<const float4*>(x);
    const float4* wv = reinterpret_cast<const float4*>(w);
    for (int q = 0; q < n4; ++q) {
        const float4 xa = xv[q], wa = wv[q];
        s0 = s0 + xa.x * wa.x;
        s1 = s1 + xa.y * wa.y;
        s2 = s2 + xa.z * wa.z;
        s3 = s3 + xa.w * wa.w;
    }
    return (s0 + s1) + (s2 + s3);
}

// optax.adam (scale_by_adam + scale(-lr)) + apply_updates, term by term:
// mu = (1-b1) g + b1 mu; nu = (1-b2) g^2 + b2 nu; u = (mu / bc1) / (sqrt(nu / bc2)
// + eps); p + u * (-lr).
__device__ __forceinline__ float dq_adam(const LearnArgs& a, float p, float g, float* __restrict__ m,
                                         float* __restrict__ v, float bc1, float bc2) {
    const float mn = a.c1 * g + a.b1 * *m;
    const float vn = a.c2 * (g * g) + a.b2 * *v;
    *m = mn;
    *v = vn;
    const float u = (mn / bc1) / (__builtin_sqrtf(vn / bc2) + a.adam_eps);
    return p + u * a.neg_lr;
}

// optax.incremental_update(new, old, tau) = tau * new + (1 - tau) * old
__device__ __forceinline__ float dq_blend(const LearnArgs& a, float nw, float old) {
    return a.tau * nw + a.one_minus_tau * old;
}

// The end of a learner step (the last workgroup, or the one workgroup of a
// step without a sample): the bias half of the target blend, then thread 0
// writes the counters and the plan drl_dqn_update_kernel reads.
__device__ void dq_finish(const LearnArgs& a, int32_t step, int trained, float loss, float bc1, float bc2) {
    const bool due = step % a.target_every == 0;
    if (due) {
        for (int l = 0; l < a.n_layers; ++l)
            for (int j = threadIdx.x; j < a.out[l]; j += blockDim.x) {
                const int64_t bi = a.boff[l] + j;
                a.target[bi] = dq_blend(a, a.online[bi], a.target[bi]);
            }
    }
    if (threadIdx.x == 0) {
        DqnCounters* c = a.ctr;
        if (trained) {
            c->count = c->count + 1;
            c->beta1_pow = c->beta1_pow * a.b1d;
            c->beta2_pow = c->beta2_pow * a.b2d;
        }
        c->loss = trained ? loss : 0.0f;
        float eps = c->epsilon;
        if (step % a.eps_every == 0) {
            const float d = eps * a.eps_decay;
            eps = d > a.eps_end ? d : a.eps_end;  // jnp.maximum
        }
        c->epsilon = eps;
        c->trained = trained;
        c->target_due = due ? 1 : 0;
        c->bc1 = bc1;
        c->bc2 = bc2;
        c->step = step + 1;
    }
}

// Copy n words src(i) -> dst(i) with every thread holding DQN_STAGE loads in
// flight before its first store (a loop with one dependent load per
// iteration would serialise them: one L2/HBM round trip each).
template <class Src, class Dst>
__device__ __forceinline__ void dq_stage(int n, Src src, Dst dst) {
    const int nt = blockDim.x;
    for (int base = threadIdx.x; base < n; base += DQN_STAGE * nt) {
        float v[DQN_STAGE];
#pragma unroll
        for (int q = 0; q < DQN_STAGE; ++q) {
            const int i = base + q * nt;
            v[q] = i < n ? src(i) : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < DQN_STAGE; ++q) {
            const int i = base + q * nt;
            if (i < n) dst(i, v[q]);
        }
    }
}

// Layer l's weights of one net -> LDS, rows padded to in + 4 floats (float4
// rows whose starts fall on different banks).
__device__ __forceinline__ void dq_stage_w(const LearnArgs& a, const float* P, int l, float* Ws) {
    const int li = a.in[l], lo = a.out[l], ls = li + 4;
    const float* src = P + a.woff[l];
    dq_stage(li * lo, [&](int i) { return src[i]; }, [&](int i, float v) { Ws[(i / li) * ls + (i % li)] = v; });
}

}  // namespace

__global__ void __launch_bounds__(DQN_THREADS) drl_dqn_grad_kernel(LearnArgs a) {
    extern __shared__ float4 dq_lds4[];
    float* lds = reinterpret_cast<float*>(dq_lds4);
    __shared__ int64_t s_idx[DQN_MAX_BATCH];
    __shared__ float s_d[DQN_MAX_BATCH], s_mx[DQN_MAX_BATCH], s_q[DQN_MAX_BATCH * 8];
    __shared__ int s_act[DQN_MAX_BATCH];
    __shared__ int s_last;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int B = a.batch, L = a.n_layers;
    // every workgroup reads the step before it arrives; the last one writes it
    const int32_t step = a.ctr->step;
    if (!a.trained) {  // buffer.can_sample is false: no train_step this step (loss 0)
        dq_finish(a, step, 0, 0.0f, 0.0f, 0.0f);
        return;
    }
    // ---- layer 0 of one net for DQN_TILE units (all workgroups)
    const int net = blockIdx.x / a.tiles0, u0 = (blockIdx.x % a.tiles0) * DQN_TILE;
    const int in = a.in[0], in4 = a.in4, out0 = a.out[0];
    const int nu = min(DQN_TILE, out0 - u0);
    if (tid < B) s_idx[tid] = dq_sample(a.seed, step, tid, a.size);
    __syncthreads();
    float* X = lds;                // [B][in4] the sampled rows (obs for the online net, next_obs for the target)
    float* Wt = lds + B * in4;     // [DQN_TILE][in4] this tile's layer-0 weight rows
    const uint32_t* rows = net ? a.r_next : a.r_obs;
    const int rw = (int)a.row_words;
    const float* P = net ? a.target : a.online;
    // this tile's weight rows are contiguous in the set: one flat copy
    const float* wsrc = P + a.woff[0] + (int64_t)u0 * in;
    dq_stage(nu * in, [&](int i) { return wsrc[i]; }, [&](int i, float v) { Wt[(i / in) * in4 + (i % in)] = v; });
    if (a.code_w) {  // the B code rows -> LDS, then decoded from there
        uint32_t* R = reinterpret_cast<uint32_t*>(Wt + DQN_TILE * in4);  // [B][rw]
        dq_stage(B * rw, [&](int i) { return __uint_as_float(rows[s_idx[i / rw] * a.row_words + (i % rw)]); },
                 [&](int i, float v) { R[i] = __float_as_uint(v); });
        __syncthreads();
        for (int e = tid; e < B * in4; e += nt) {
            const int b = e / in4, k = e - b * in4;
            X[e] = k < in ? dq_input(a, R + b * rw, 0, k) : 0.0f;
        }
    } else {
        dq_stage(B * in4, [&](int i) {
            const int b = i / in4, k = i - b * in4;
            return k < in ? __uint_as_float(rows[s_idx[b] * a.row_words + k]) : 0.0f;
        }, [&](int i, float v) { X[i] = v; });
    }
    for (int e = tid; e < (DQN_TILE - nu) * in4; e += nt) Wt[nu * in4 + e] = 0.0f;  // (a partial last tile)
    __syncthreads();
    if (net == 0 && u0 == 0)  // the update kernel's layer-0 inputs
        for (int e = tid; e < B * in4; e += nt) a.sx[e] = X[e];
    for (int o = tid; o < DQN_TILE * B; o += nt) {
        const int u = o % DQN_TILE, b = o / DQN_TILE;
        if (u < nu) {
            const float z = dq_dot(X + b * in4, Wt + u * in4, in4 / 4) + P[a.boff[0] + u0 + u];
            a.sz0[((int64_t)net * B + b) * out0 + u0 + u] = z;
        }
    }
    // publish: stores drained, one agent-scope release, the ticket; the last
    // arriver acquires (cdna_hip_programming.md §5 split-K recipe)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int t = __hip_atomic_fetch_add(&a.ctr->arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (t == a.nblk0 - 1);
    }
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&a.ctr->arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();

    // ---- the last workgroup: later layers (one net at a time, each layer's
    // weights staged in LDS), TD error, backward, biases
    const int mw = a.maxw;
    float* Pa = lds;                   // [B][mw] activations of the current layer
    float* Qa = lds + B * mw;          // [B][mw] the next layer's
    float* Ws = lds + 2 * B * mw;      // one layer's weights, rows of in + 4 floats
    uint8_t* M = reinterpret_cast<uint8_t*>(Ws + a.ws_floats);  // [L-1][B][mw] online ReLU masks (z > 0)
    const int A = a.out[L - 1];
    for (int n = 1; n >= 0; --n) {  // the target net on next_obs, then the online net on obs
        const float* Pn = n ? a.target : a.online;
        dq_stage(B * out0, [&](int i) { return a.sz0[(int64_t)n * B * out0 + i]; }, [&](int i, float z) {
            const int b = i / out0, j = i - b * out0;
            const float h = z > 0.0f ? z : 0.0f;
            Pa[b * mw + j] = h;
            if (n == 0) {
                a.sh[0][i] = h;
                M[b * mw + j] = z > 0.0f;
            }
        });
        for (int l = 1; l < L; ++l) {
            const int li = a.out[l - 1], lo = a.out[l], ls = li + 4;
            const bool hidden = l < L - 1;
            dq_stage_w(a, Pn, l, Ws);
            __syncthreads();
            for (int o = tid; o < B * lo; o += nt) {
                const int b = o / lo, j = o - b * lo;
                const float z = dq_dot(Pa + b * mw, Ws + j * ls, li / 4) + Pn[a.boff[l] + j];
                if (hidden) {
                    const float h = z > 0.0f ? z : 0.0f;
                    Qa[b * mw + j] = h;
                    if (n == 0) {
                        a.sh[l][o] = h;
                        M[(l * B + b) * mw + j] = z > 0.0f;
                    }
                } else {
                    Qa[b * mw + j] = z;
                }
            }
            __syncthreads();
            float* t = Pa;
            Pa = Qa;
            Qa = t;
        }
        // Pa: the net's Q [B][A]
        for (int b = tid; b < B; b += nt) {
            if (n == 1) {
                float mx = Pa[b * mw];
                for (int j = 1; j < A; ++j) mx = Pa[b * mw + j] > mx ? Pa[b * mw + j] : mx;  // jnp.max
                s_mx[b] = mx;
            } else {
                for (int j = 0; j < A; ++j) s_q[b * 8 + j] = Pa[b * mw + j];
            }
        }
        __syncthreads();
    }
    // Ws still holds the online net's output layer (the first backward step's weights)
    for (int b = tid; b < B; b += nt) {
        const int64_t s = s_idx[b];
        const int act = a.r_act[s];
        const float notdone = a.r_done[s] ? 0.0f : 1.0f;
        const float td = a.r_rew[s] + (a.gamma * s_mx[b]) * notdone;
        const bool ok = act >= 0 && act < A;
        s_d[b] = (ok ? s_q[b * 8 + act] : td) - td;  // (an action outside [0, A) adds nothing)
        s_act[b] = ok ? act : -1;
    }
    __syncthreads();
    float loss = 0.0f;
    for (int b = 0; b < B; ++b) loss = loss + s_d[b] * s_d[b];
    loss = loss / (float)B;  // jnp.mean(jnp.square(q - td))
    // d loss / d q[b][a_b] = 2 (q - td) / B: the output layer's deltas
    float* D = Pa;   // [B][mw] deltas of layer l
    float* D2 = Qa;  // [B][mw] deltas of layer l - 1
    for (int o = tid; o < B * A; o += nt) {
        const int b = o / A, j = o - b * A;
        const float dq = (s_act[b] == j) ? (s_d[b] + s_d[b]) / (float)B : 0.0f;
        D[b * mw + j] = dq;
        a.sd[L - 1][o] = dq;
    }
    __syncthreads();
    // Adam's bias corrections for this step (count + 1): 1 - beta^count in double, rounded once
    const double p1 = a.ctr->beta1_pow * a.b1d, p2 = a.ctr->beta2_pow * a.b2d;
    const float bc1 = (float)(1.0 - p1), bc2 = (float)(1.0 - p2);
    for (int l = L - 1; l >= 0; --l) {
        const int lo = a.out[l];
        for (int j = tid; j < lo; j += nt) {  // the bias: sum of the deltas over the batch, Adam
            float g = 0.0f;
            for (int b = 0; b < B; ++b) g = g + D[b * mw + j];
            const int64_t bi = a.boff[l] + j;
            a.online[bi] = dq_adam(a, a.online[bi], g, a.adam_m + bi, a.adam_v + bi, bc1, bc2);
        }
        if (l == 0) break;
        const int li = a.out[l - 1], ls = li + 4;
        if (l < L - 1) {  // (W_{L-1} is still staged from the forward pass)
            __syncthreads();
            dq_stage_w(a, a.online, l, Ws);  // (this step's weights: the update kernel writes them next)
            __syncthreads();
        }
        for (int o = tid; o < B * li; o += nt) {
            const int b = o / li, i = o - b * li;
            float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int j = 0; j < lo; ++j) s4[j & 3] = s4[j & 3] + D[b * mw + j] * Ws[j * ls + i];
            const float dz = M[((l - 1) * B + b) * mw + i] ? (s4[0] + s4[1]) + (s4[2] + s4[3]) : 0.0f;
            D2[b * mw + i] = dz;
            a.sd[l - 1][o] = dz;
        }
        __syncthreads();
        float* t = D;
        D = D2;
        D2 = t;
    }
    __syncthreads();  // (the bias updates are read by the target blend)
    dq_finish(a, step, 1, loss, bc1, bc2);
}

// One thread per element of the packed net (hi fragments, then biases).
__global__ void __launch_bounds__(256) drl_dqn_update_kernel(LearnArgs a) {
    const int trained = a.ctr->trained, due = a.ctr->target_due;
    if (!trained && !due) return;
    const QnetPack& p = a.pack;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < p.n_wfrag_elems) {
        int l = 0;
        while (l + 1 < p.n_layers && i >= (int64_t)p.frag_src[l + 1] * 8) ++l;
        const int64_t e = i - (int64_t)p.frag_src[l] * 8;
        const PackSlot s = qnet_pack_slot(l, e, p.kt[l], p.code_w, p.in[l]);
        if (s.row >= p.out[l]) return;
        if (s.k < 0) {  // a code net's layer-0 bias slot: the bias the gradient kernel updated
            if (trained) qnet_pack_write(p, l, e, -1, a.online[a.boff[0] + s.row]);
            return;
        }
        if (s.k >= p.in[l]) return;
        const int64_t wi = a.woff[l] + (int64_t)s.row * p.in[l] + s.k;
        float w = a.online[wi];
        if (trained) {
            const float* D = a.sd[l] + s.row;
            const float* X = (l ? a.sh[l - 1] : a.sx) + s.k;
            const int xs = l ? p.in[l] : a.in4, ds = p.out[l];
            const float m0 = a.adam_m[wi], v0 = a.adam_v[wi];
            // the batch sum in row order, DQN_STAGE rows' operands loaded ahead
            float g = 0.0f;
            for (int b0 = 0; b0 < a.batch; b0 += DQN_STAGE) {
                float dv[DQN_STAGE], xv[DQN_STAGE];
#pragma unroll
                for (int q = 0; q < DQN_STAGE; ++q) {
                    const int b = b0 + q < a.batch ? b0 + q : a.batch - 1;
                    dv[q] = D[b * ds];
                    xv[q] = X[b * xs];
                }
#pragma unroll
                for (int q = 0; q < DQN_STAGE; ++q)
                    if (b0 + q < a.batch) g = g + dv[q] * xv[q];
            }
            float m = m0, v = v0;
            w = dq_adam(a, w, g, &m, &v, a.ctr->bc1, a.ctr->bc2);
            a.adam_m[wi] = m;
            a.adam_v[wi] = v;
            a.online[wi] = w;
            qnet_pack_write(p, l, e, s.k, w);
        }
        if (due) a.target[wi] = dq_blend(a, w, a.target[wi]);
    } else if (i < p.n_wfrag_elems + p.n_bias) {
        if (!trained) return;
        const int64_t bi = i - p.n_wfrag_elems;
        int l = 0;
        while (l + 1 < p.n_layers && bi >= p.bias_off[l + 1]) ++l;
        const int u = (int)(bi - p.bias_off[l]);
        if (u < p.out[l]) p.packed_b[bi] = a.online[a.boff[l] + u];
    }
}

__global__ void drl_dqn_init_kernel(DqnCounters* c, float epsilon) {
    if (threadIdx.x == 0) {
        c->step = 0;
        c->count = 0;
        c->epsilon = epsilon;
        c->loss = 0.0f;
        c->beta1_pow = 1.0;
        c->beta2_pow = 1.0;
        c->arrive = 0;
        c->trained = 0;
        c->target_due = 0;
        c->bc1 = 0.0f;
        c->bc2 = 0.0f;
        c->pad[0] = c->pad[1] = c->pad[2] = 0;
    }
}

hipError_t launch_dqn_train(const LearnArgs& a, size_t lds_grad, hipStream_t s) {
    if (a.trained)
        hipLaunchKernelGGL(drl_dqn_grad_kernel, dim3((unsigned)a.nblk0), dim3(DQN_THREADS), lds_grad, s, a);
    else
        hipLaunchKernelGGL(drl_dqn_grad_kernel, dim3(1), dim3(DQN_THREADS), 0, s, a);
    const int64_t n = a.pack.n_wfrag_elems + a.pack.n_bias;
    hipLaunchKernelGGL(drl_dqn_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dqn_init(void* counters, float epsilon, hipStream_t s) {
    hipLaunchKernelGGL(drl_dqn_init_kernel, dim3(1), dim3(64), 0, s, static_cast<DqnCounters*>(counters), epsilon);
    return hipGetLastError();
}

}  // namespace drl
