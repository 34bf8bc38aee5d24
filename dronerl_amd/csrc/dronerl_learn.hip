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
// One launch (drl_dqn_train_kernel) per learner step: workgroups split
// layer 0 of both nets (online on the sampled obs, target on next_obs) in
// DQN_TILE-unit tiles and hand their pre-activations over with write-through
// stores and a ticket counter; two more workgroups (the tails, one per net)
// prefetch everything else into LDS meanwhile, wait for the tickets, and run
// their net's later layers; the online tail then runs the TD error, the loss
// and the backward pass down to layer 1's deltas and hands them over behind
// an epoch word, on which the layer-0 workgroups update the weights (their
// own layer-0 deltas, gradient, Adam, the act kernels' packed fp16 hi/lo or
// bf16 image, the target blend) while the online tail updates the biases.
//
// Arithmetic order is fixed and contraction-free (each product rounded, then
// each sum), so oracle/dqn_learner.py reproduces the result bit for bit:
// a dot product of length n keeps four partial sums over k mod 4, each in k
// order, combined (s0 + s1) + (s2 + s3), then + bias (dq_mm: one lane per
// partial sum); a batch sum runs over rows in order; Adam is optax's formula
// term by term.  The f32 constants are
// what jax's weak typing makes of the python floats (1 - b1 rounded once).
// The learner is latency-bound (a batch of 8 rows): VALU, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronerl_internal.h"

// every product and sum of this file rounds on its own (no FMA contraction): the order oracle/dqn_learner.py restates
#pragma clang fp contract(off)

namespace drl {

// DRL_DQN_STAMPS (diagnostic builds, tools/learn_stamps.py): thread 0 of each
// workgroup stores wall_clock64() (100 MHz) at phase boundaries (16 slots each) into the 8 KB
// the layout appends to the agent block's scratch.
#ifdef DRL_DQN_STAMPS
#define DQ_STAMP(i) \
    do { if (threadIdx.x == 0) a.stamps[16 * blockIdx.x + (i)] = wall_clock64(); } while (0)
#else
#define DQ_STAMP(i) do { } while (0)
#endif

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

// The counters at the end of a learner step (thread 0 of the online tail,
// or of the one workgroup of a step without a sample): Adam's count and
// powers, the loss, the epsilon decay, the step's plan (informative),
// step + 1.  ctr: the values the kernel read at its start.
__device__ void dq_finish(const LearnArgs& a, const DqnCounters& ctr, int trained, float loss, float bc1, float bc2) {
    if (threadIdx.x != 0) return;
    DqnCounters* c = a.ctr;
    const int32_t step = ctr.step;
    if (trained) {
        c->count = ctr.count + 1;
        c->beta1_pow = ctr.beta1_pow * a.b1d;
        c->beta2_pow = ctr.beta2_pow * a.b2d;
    }
    c->loss = trained ? loss : 0.0f;
    float eps = ctr.epsilon;
    if (step % a.eps_every == 0) {
        const float d = eps * a.eps_decay;
        eps = d > a.eps_end ? d : a.eps_end;  // jnp.maximum
    }
    c->epsilon = eps;
    c->trained = trained;
    c->target_due = step % a.target_every == 0 ? 1 : 0;
    c->bc1 = bc1;
    c->bc2 = bc2;
    c->step = step + 1;
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

// Layer l's weights of one net -> LDS, rows padded to in + 4 floats (in is a
// multiple of 32: consecutive rows of a micro-tile start 4 banks apart).
__device__ __forceinline__ void dq_stage_w(const LearnArgs& a, const float* P, int l, float* Ws) {
    const int li = a.in[l], lo = a.out[l], ls = li + 4;
    const float* src = P + a.woff[l];
    dq_stage(li * lo, [&](int i) { return src[i]; }, [&](int i, float v) { Ws[(i / li) * ls + (i % li)] = v; });
}

typedef const __attribute__((address_space(1))) float gcf32;
typedef float dq_f4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) dq_f4 gcf4;
typedef float dq_f2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) dq_f2 gcf2;
typedef const __attribute__((address_space(1))) uint8_t gcu8;

__device__ __forceinline__ uint32_t dq_div(uint32_t i, const DqSeg& g) { return g.rm ? __umulhi(i, g.rm) : i; }

// (global-address-space loads: a flat load would also count against the LDS counter)
typedef const void* dq_tab[5][DQN_MAX_BATCH];  // the sampled rows' obs, next_obs, action, reward, done pointers
__device__ __forceinline__ dq_f4 dq_seg_load(const DqSeg& g, int i, const dq_tab& tab) {
    switch (g.kind) {
        case 0: return dq_f4{((gcf32*)g.src)[i], 0.0f, 0.0f, 0.0f};
        case 1: return dq_f4{*(gcf32*)tab[g.tbl][i], 0.0f, 0.0f, 0.0f};
        case 2: return dq_f4{*(gcu8*)tab[4][i] ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f};
        case 3: {
            const int b = (int)dq_div((uint32_t)i, g);
            return dq_f4{((gcf32*)tab[g.tbl][b])[i - b * g.row], 0.0f, 0.0f, 0.0f};
        }
        case 5: {
            const dq_f2 v = ((gcf2*)g.src)[i];
            return dq_f4{v.x, v.y, 0.0f, 0.0f};
        }
        default: return ((gcf4*)g.src)[i];
    }
}
__device__ __forceinline__ int dq_seg_width(const DqSeg& g) { return g.kind == 4 ? 4 : g.kind == 5 ? 2 : 1; }
__device__ __forceinline__ int dq_seg_dst(const DqSeg& g, int i) {
    const int w = dq_seg_width(g);
    if (!g.pad) return g.dst + w * i;
    const int r = (int)dq_div((uint32_t)i, g), c = i - r * g.row;
    return g.dst + w * (r * (g.row + g.pad) + c);
}

// The segments seg[0..ns) (start: their prefix sums, start[ns] = total) in
// one pass: DQN_STAGE loads per thread in flight, then their LDS stores.  A
// thread's elements only move forward, so its segment is carried in
// registers and re-read from LDS only when it crosses into the next one.
__device__ __forceinline__ void dq_stage_segs(float* lds, const DqSeg* seg, const int* start, int ns,
                                              const dq_tab& tab) {
    const int n = start[ns], nt = blockDim.x;  // (start[0] may be > 0: a later part of a list)
    int g = 0, ge = start[1], gs = start[0];
    DqSeg cur = seg[0];
    for (int base = start[0] + threadIdx.x; base < n; base += DQN_STAGE * nt) {
        dq_f4 v[DQN_STAGE];
        int d[DQN_STAGE];
        int w4[DQN_STAGE];
#pragma unroll
        for (int q = 0; q < DQN_STAGE; ++q) {
            const int i = base + q * nt;
            d[q] = -1;
            w4[q] = 1;
            if (i < n) {
                while (i >= ge) {
                    ++g;
                    cur = seg[g];
                    gs = ge;
                    ge = start[g + 1];
                }
                v[q] = dq_seg_load(cur, i - gs, tab);
                d[q] = dq_seg_dst(cur, i - gs);
                w4[q] = dq_seg_width(cur);
            }
        }
#pragma unroll
        for (int q = 0; q < DQN_STAGE; ++q) {
            if (d[q] < 0) continue;
            if (w4[q] == 4) *reinterpret_cast<dq_f4*>(lds + d[q]) = v[q];
            else if (w4[q] == 2) *reinterpret_cast<dq_f2*>(lds + d[q]) = dq_f2{v[q].x, v[q].y};
            else lds[d[q]] = v[q].x;
        }
    }
}

// Write-through (sc1) store / load of a handed-off word (MI355X_MICROARCH.md
// § visibility, Valid forms, table row 1: every store and every load of the
// bytes sc1; the consumer polls the one agent-scope counter with sc1 loads).
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ void dq_store_sc1(float* p, float v) {
    __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float dq_load_sc1(const float* p) {
    return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Granule hand-off (MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16, R2: the data is the flag):
// one naturally aligned 8-byte {tag = epoch, value} written by one sc1 store; the reader polls it with sc1
// loads until the tag is this step's epoch (never 0; drl_dqn_init zeroes the scratch).  No ticket, no drain.
// A launch that gave up on a hand-off leaves pad[0] set, and every later launch then returns at once (see
// the kernel's entry), so a stale granule of an aborted step (same epoch: step did not advance) is never read.
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ void dq_granule_put(uint64_t* g, uint32_t epoch, float v) {
    __hip_atomic_store((gu64*)g, ((uint64_t)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// false after a bounded wait (DqnCounters::pad[0] = 1)
__device__ __forceinline__ bool dq_granule_get(const LearnArgs& a, const uint64_t* g, uint32_t epoch, float* v) {
    for (uint32_t spins = 0;; ++spins) {
        const uint64_t x = __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(x >> 32) == epoch) {
            *v = __uint_as_float((uint32_t)x);
            return true;
        }
        if (spins > a.spin_granule) {
            a.ctr->pad[0] = 1;
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// 16-B write-through stores and loads (buffer ops, aux 16 = sc1: the same hand-off form as the 4-B ones, at
// one fabric write per 16 B instead of per 4 B: MI355X_MICROARCH.md § visibility, stores of each flavour).
typedef unsigned dq_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dq_rsrc(const float* p, int nfloats) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, nfloats * 4, 0x00020000);
}
// rows b < B of an LDS buffer (stride ss, the first n floats, n % 4 == 0) -> global rows of stride ds
__device__ __forceinline__ void dq_publish(const float* src, int ss, float* dst, int ds, int B, int n) {
    const __amdgpu_buffer_rsrc_t r = dq_rsrc(dst, (B - 1) * ds + n);
    const int n4 = n >> 2;
    for (int i = threadIdx.x; i < B * n4; i += blockDim.x) {
        const int b = i / n4, j = 4 * (i - b * n4);
        const dq_f4 v = *reinterpret_cast<const dq_f4*>(src + b * ss + j);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dq_u4, v), r, (b * ds + j) * 4, 0, 16);
    }
}

// The learner's dot products as micro-tiles: z[b][j] = sum over k < n of
// X[b * xs + k * xk] * W[j * wr + k * wk] for b < B, j < J.  A group of four
// lanes takes two rows b by two outputs j; lane c of the group accumulates
// the partial sums of k = c (mod 4) in k order -- exactly the canonical four
// partial sums -- and the group combines them as (s0 + s1) + (s2 + s3) by
// lane swaps (float addition commutes, so every lane holds the same value).
// out(b, j, z) runs once per output, on lane c == 0.  Every lane of a wave
// runs every iteration (the swaps need the whole wave).
template <class Out>
__device__ __forceinline__ void dq_mm(const float* X, int xs, int xk, const float* W, int wr, int wk, int n, int B,
                                      int J, Out out) {
    const int nbp = (B + 1) / 2, njp = (J + 1) / 2, items = nbp * njp * 4;
    for (int base = 0; base < items; base += blockDim.x) {
        const int it = base + threadIdx.x;
        const bool live = it < items;
        const int c = it & 3, pr = it >> 2;
        const int jp = pr % njp, bp = pr / njp;
        const int b0 = 2 * bp, b1 = min(b0 + 1, B - 1), j0 = 2 * jp, j1 = min(j0 + 1, J - 1);
        float s00 = 0.0f, s01 = 0.0f, s10 = 0.0f, s11 = 0.0f;
        if (live) {
            const float *x0 = X + b0 * xs, *x1 = X + b1 * xs, *w0 = W + j0 * wr, *w1 = W + j1 * wr;
#pragma unroll 4
            for (int k = c; k < n; k += 4) {
                const float a0 = x0[k * xk], a1 = x1[k * xk], c0 = w0[k * wk], c1 = w1[k * wk];
                s00 = s00 + a0 * c0;
                s01 = s01 + a0 * c1;
                s10 = s10 + a1 * c0;
                s11 = s11 + a1 * c1;
            }
        }
        s00 = s00 + __shfl_xor(s00, 1);
        s01 = s01 + __shfl_xor(s01, 1);
        s10 = s10 + __shfl_xor(s10, 1);
        s11 = s11 + __shfl_xor(s11, 1);
        s00 = s00 + __shfl_xor(s00, 2);
        s01 = s01 + __shfl_xor(s01, 2);
        s10 = s10 + __shfl_xor(s10, 2);
        s11 = s11 + __shfl_xor(s11, 2);
        if (live && c == 0) {
            out(b0, j0, s00);
            if (j1 != j0) out(b0, j1, s01);
            if (b1 != b0) {
                out(b1, j0, s10);
                if (j1 != j0) out(b1, j1, s11);
            }
        }
    }
}

// The same dot products with one output per lane quad (lane c: k = c mod 4):
// four times the lanes of dq_mm and a quarter of its per-lane chain, for
// the layer-0 workgroups' small output tiles (DQN_TILE units x B rows).
template <class Out>
__device__ __forceinline__ void dq_mm1(const float* X, int xs, const float* W, int wr, int wk, int n, int B, int J,
                                       Out out) {
    const int items = B * J * 4;
    for (int base = 0; base < items; base += blockDim.x) {
        const int it = base + threadIdx.x;
        const bool live = it < items;
        const int c = it & 3, pr = it >> 2;
        const int j = pr % J, b = pr / J;
        float s = 0.0f;
        if (live) {
            const float *x = X + b * xs, *w = W + j * wr;
#pragma unroll 8
            for (int k = c; k < n; k += 4) s = s + x[k] * w[k * wk];
        }
        s = s + __shfl_xor(s, 1);
        s = s + __shfl_xor(s, 2);
        if (live && c == 0) out(b, j, s);
    }
}

// The later layers of net n (1 = target, 0 = online) for the B sampled rows,
// from its layer-0 pre-activations (handed over write-through) and its
// prefetched (or staged) weights; returns the buffer holding Q [B][A].  The
// online net also hands its hidden activations over (write-through: the
// update phase reads them) and keeps its ReLU masks in LDS.
__device__ __forceinline__ float* dq_forward(const LearnArgs& a, int n, float* Pa, float* Qa, float* Ws, uint8_t* M,
                                             const float* T, uint32_t epoch, int* ok) {
    const int B = a.batch, L = a.n_layers, mw = a.maxw, out0 = a.out[0];
    const float* Pn = n ? a.target : a.online;
    // the layer-0 workgroups' pre-activations: each thread polls its granules until they carry this epoch
    const uint64_t* g = a.gz0 + (int64_t)n * B * out0;
    for (int e = threadIdx.x; e < B * out0; e += blockDim.x) {
        float z;
        if (!dq_granule_get(a, g + e, epoch, &z)) {
            *ok = 0;
            break;
        }
        const int b = e / out0, j = e - b * out0;
        Pa[b * mw + j] = z > 0.0f ? z : 0.0f;
        if (n == 0) M[b * mw + j] = z > 0.0f;
    }
    __syncthreads();
    if (!*ok) return nullptr;
    DQ_STAMP(8);
    if (n == 0) dq_publish(Pa, mw, a.sh[0], out0, B, out0);
    for (int l = 1; l < L; ++l) {
        // (prefetched rows: in + 2 floats, = 2 mod 32 for in a multiple of 32: the micro-tiles' two rows
        // and four k classes hit 64 different banks; staged rows: in + 4)
        const int li = a.out[l - 1], lo = a.out[l], ls = li + (a.prefetch ? 2 : 4);
        const bool hidden = l < L - 1;
        const float* W = a.prefetch ? T + a.tw[n][l] : Ws;
        const float* bias = T + a.tb[n][l];
        if (!a.prefetch) dq_stage_w(a, Pn, l, Ws);
        __syncthreads();
        auto put = [&](int b, int j, float d) {
            const float z = d + bias[j];
            if (hidden) {
                Qa[b * mw + j] = z > 0.0f ? z : 0.0f;
                if (n == 0) M[(l * B + b) * mw + j] = z > 0.0f;
            } else {
                Qa[b * mw + j] = z;
            }
        };
        if (lo <= 8)  // (the 5-action output layer: one output per quad, more lanes, a shorter chain each)
            dq_mm1(Pa, mw, W, ls, 1, li, B, lo, put);
        else
            dq_mm(Pa, mw, 1, W, ls, 1, li, B, lo, put);
        __syncthreads();
        DQ_STAMP(8 + l);
        if (n == 0 && hidden) dq_publish(Qa, mw, a.sh[l], lo, B, lo);
        float* t = Pa;
        Pa = Qa;
        Qa = t;
    }
    return Pa;
}

// Poll an agent-scope word (sc1 loads, one lane) until it reaches `want`;
// false after a bounded wait (DqnCounters::pad[0] = 1).
__device__ __forceinline__ bool dq_wait(const LearnArgs& a, int32_t* word, uint32_t want) {
    uint32_t spins = 0;
    while (__hip_atomic_load((gu32*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > a.spin_word) {
            a.ctr->pad[0] = 1;
            return false;
        }
    }
    return true;
}

// The weight step of DQN_UB weights at a time (their loads issued together):
// gradient g[q] (the caller's batch sum), Adam, the act kernels' packed
// image (qnet_pack_elem), the target blend when due.
struct DqW {
    int l, row, k;
    int64_t wi;
    float g;
};
__device__ __forceinline__ void dq_update_weights(const LearnArgs& a, const DqW (&w)[DQN_UB], int cnt, float bc1,
                                                  float bc2, bool due) {
    float p[DQN_UB], m[DQN_UB], v[DQN_UB], t[DQN_UB];
    uint32_t px[DQN_UB];
#pragma unroll
    for (int q = 0; q < DQN_UB; ++q) {
        const int64_t wi = q < cnt ? w[q].wi : w[0].wi;
        p[q] = a.online[wi];
        m[q] = a.adam_m[wi];
        v[q] = a.adam_v[wi];
        px[q] = a.pidx[wi];
        t[q] = due ? a.target[wi] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < DQN_UB; ++q) {
        if (q >= cnt) break;
        const float nw = dq_adam(a, p[q], w[q].g, &m[q], &v[q], bc1, bc2);
        a.online[w[q].wi] = nw;
        a.adam_m[w[q].wi] = m[q];
        a.adam_v[w[q].wi] = v[q];
        qnet_pack_write_idx(a.pack, w[q].l, px[q], nw);
        if (due) a.target[w[q].wi] = dq_blend(a, nw, t[q]);
    }
}

}  // namespace

// One launch per learner step.  Workgroup 0 is the online tail, 1 the target
// tail, 2 .. 2 + nblk0 - 1 the layer-0 workgroups (net = (w - 2) / tiles0):
//  1. layer-0 workgroups: their net's layer 0 for DQN_TILE units on the
//     sampled rows, handed over write-through behind one ticket each; the
//     tails prefetch their net's later layers (the online tail also the
//     biases, their moments and the rows' action / reward / done) meanwhile;
//  2. the target tail: the target net's later layers, max_a Q_target handed
//     over; the online tail: the online net's later layers, the TD error, the
//     loss, the backward pass to layer 1's deltas, handed over with the hidden
//     activations behind an epoch word; then layer 0's deltas and the bias
//     updates (Adam, packed image, target blend), the counters;
//  3. the layer-0 workgroups take the weights: the online ones form their
//     units' layer-0 deltas and update their layer-0 rows (inputs still in
//     LDS), the target ones a share of the later layers: gradient, Adam,
//     packed image, target blend.
// The tails are workgroups 0 and 1 so that they are dispatched first: every
// wait in the kernel is on work that is already running.
// TRAINED: the launch's plan (host-known: size >= batch) as a template parameter, so the trained instance has
// no branch at its top that the compiler could sink the weight tile's loads below (they go out first)
template <bool TRAINED>
__global__ void __launch_bounds__(DQN_THREADS) drl_dqn_train_kernel(LearnArgs args) {
    // the arguments read in place from the kernarg segment (a by-value parameter that inlined code takes
    // references to can be copied into private memory: 2.4 KB of scratch traffic per workgroup)
    (void)args;
    const LearnArgs& a = *(const LearnArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    extern __shared__ float4 dq_lds4[];
    float* lds = reinterpret_cast<float*>(dq_lds4);
    __shared__ dq_tab s_tab;
    __shared__ float s_d[DQN_MAX_BATCH], s_mx[DQN_MAX_BATCH], s_q[DQN_MAX_BATCH * 8];
    __shared__ float s_gb[QN_MAX_LAYERS][128];  // (online tail) the biases' gradients, formed with the deltas
    __shared__ int s_act[DQN_MAX_BATCH];
    __shared__ DqSeg s_seg[DQN_MAX_SEGS];
    __shared__ int s_start[DQN_MAX_SEGS + 1];
    __shared__ int s_flag;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int B = a.batch, L = a.n_layers;
    // a layer-0 workgroup's weight tile does not depend on the counters: its loads go out first, beside the
    // counters' (up to DQN_W0R per thread in registers; the rest, for inputs above 512, staged below)
    const int in = a.in[0], in4 = a.in4, xs0 = a.xs0, out0 = a.out[0];
    const int w0 = blockIdx.x - 2, net0 = w0 / (a.tiles0 > 0 ? a.tiles0 : 1);
    const int u00 = (w0 % (a.tiles0 > 0 ? a.tiles0 : 1)) * DQN_TILE, nu0 = min(DQN_TILE, out0 - u00);
    const bool l0wg = TRAINED && blockIdx.x >= 2;
    const int nw0 = l0wg ? nu0 * in : 0;
    float w0r[DQN_W0R];
    {
        // unconditional loads at clamped indices (no exec-mask branch around them, so the counters' wait stays
        // vmcnt(DQN_W0R) instead of vmcnt(0)); the tails read the online set's first float and discard it
        const float* src = l0wg ? (net0 ? a.target : a.online) + a.woff[0] + (int64_t)u00 * in : a.online;
#pragma unroll
        for (int q = 0; q < DQN_W0R; ++q) {
            const int e = threadIdx.x + q * DQN_THREADS;
            const float v = ((gcf32*)src)[e < nw0 ? e : 0];
            w0r[q] = e < nw0 ? v : 0.0f;
        }
    }
    // the counters as this step starts (the online tail writes them at the end): scalar loads (lgkmcnt), so
    // the sample -> row-pointer chain below waits for them only, not for the weight tile issued before them
    // (vmcnt), whose LDS store now follows the rows' staging
    DqnCounters ctr;
    // (a learner whose block carries the timeout flag does nothing until drl_dqn_init clears it: the aborted
    // launch left granules tagged with this step's epoch and the arrive ticket part-counted.  Each path returns
    // before its first global write or hand-off; no early branch here, where the compiler would sink the weight
    // loads above below it, behind this load)
    const int32_t flag = a.ctr->pad[0];
    ctr.step = a.ctr->step;
    ctr.count = a.ctr->count;
    ctr.epsilon = a.ctr->epsilon;
    ctr.beta1_pow = a.ctr->beta1_pow;
    ctr.beta2_pow = a.ctr->beta2_pow;
    const bool due = ctr.step % a.target_every == 0;
    DQ_STAMP(0);
#ifdef DRL_DQN_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the shader clock against the 100 MHz wall clock
        a.stamps[1000] = clock64();
        a.stamps[1001] = wall_clock64();
    }
#endif
    if constexpr (!TRAINED) {  // buffer.can_sample is false: no train_step this step (loss 0); the target blend when due
        if (flag != 0) return;
        if (due)
            for (int64_t i = tid; i < a.n_params; i += nt) a.target[i] = dq_blend(a, a.online[i], a.target[i]);
        dq_finish(a, ctr, 0, 0.0f, 0.0f, 0.0f);
        return;
    }
    // Adam's bias corrections for this step (count + 1): 1 - beta^count in double, rounded once
    const float bc1 = (float)(1.0 - ctr.beta1_pow * a.b1d), bc2 = (float)(1.0 - ctr.beta2_pow * a.b2d);
    if (tid < B) {  // buffers.py:79-90 sample: the rows' pointers (a pending add's rows from its own buffers)
        const int64_t s = dq_sample(a.seed, ctr.step, tid, a.size);
        const void* p[5] = {a.r_obs + s * a.row_words, a.r_next + s * a.row_words, a.r_act + s, a.r_rew + s,
                            a.r_done + s};
        if (a.fresh) {
            int64_t off = s - a.f_base;
            if (off < 0) off += a.capacity;
            if (off < a.f_rows) {
                const int64_t i = a.f_first + off;
                p[0] = a.f_obs + i * a.f_obs_stride;
                p[1] = a.f_next + i * a.f_next_stride;
                p[2] = a.f_act + i * a.f_act_stride;
                p[3] = a.f_rew + i * a.f_rew_stride;
                p[4] = a.f_done + i * a.f_done_stride;
            }
        }
        for (int t = 0; t < 5; ++t) s_tab[t][tid] = p[t];
    }
    const uint32_t epoch = (uint32_t)ctr.step + 1u;  // the online tail's hand-off word (pad[2]) for this step
    if (blockIdx.x >= 2) {
        // ---- 1. layer 0 of one net for DQN_TILE units
        const int w = blockIdx.x - 2, net = w / a.tiles0, u0 = (w % a.tiles0) * DQN_TILE;
        const int nu = min(DQN_TILE, out0 - u0);
        float* X = lds;                   // [B][in4] the sampled rows (obs: online net, next_obs: target)
        float* Wt = lds + B * in4;        // [DQN_TILE][xs0] this tile's layer-0 weight rows, then its biases
        float* Bt = Wt + DQN_TILE * xs0;
        const int rw = (int)a.row_words;
        float* Z = Bt + DQN_TILE + (a.code_w ? B * rw : 0);  // [B][DQN_TILE] the tile's pre-activations
        float* W1s = Z + B * DQN_TILE;                         // (online, L > 1) [out1][DQN_TILE + 1] W_1's columns
        float* D1s = W1s + (L > 1 ? a.out[1] * (DQN_TILE + 1) : 0);  // [B][out1] the handed-over layer-1 deltas
        const float* P = net ? a.target : a.online;
        if (tid == 0) {  // the biases, the rows (the tile's weights are in registers: in <= 512, the plan checks)
            s_seg[0] = DqSeg{P + a.boff[0] + u0, nu, B * in4 + DQN_TILE * xs0, 1, 0, 0, 0u, 0};
            if (a.code_w)  // the code rows, decoded from LDS below
                s_seg[1] = DqSeg{nullptr, B * rw, B * in4 + DQN_TILE * xs0 + DQN_TILE, rw, 0, 3, a.rm_rw, net};
            else
                s_seg[1] = DqSeg{nullptr, B * in, 0, in, in4 - in, 3, a.rm_in, net};
            s_start[0] = 0;
            s_start[1] = nu;
            s_start[2] = nu + s_seg[1].n;
        }
        for (int e = tid; e < B * (in4 - in); e += nt) X[(e / (in4 - in)) * in4 + in + e % (in4 - in)] = 0.0f;
        __syncthreads();
        DQ_STAMP(1);
        dq_stage_segs(lds, s_seg, s_start, 2, s_tab);
        // the registers' weights -> rows of xs0 (after the rows' loads are issued: the weights landed first)
#pragma unroll
        for (int q = 0; q < DQN_W0R; ++q) {
            const int e = tid + q * nt;
            if (e < nw0) {
                const int r = (int)__umulhi((uint32_t)e, a.rm_in);
                Wt[r * xs0 + (e - r * in)] = w0r[q];
            }
        }
        if (flag != 0) return;  // (uniform; nothing written or handed off yet)
        __syncthreads();
        DQ_STAMP(2);
        // the online tile's columns of W_1 (it forms its own layer-0 deltas from them, 3. below): loaded into
        // registers now, stored to LDS after the tile's dot products, and landed before this workgroup's
        // ticket (the drain below), so no read of them can see the update workgroups' writes
        constexpr int W1R = 4;  // (out1 <= 128 hidden units x 8 = 2 per thread)
        float w1r[W1R];
        const bool w1 = net == 0 && L > 1;
        const int n1 = w1 ? a.out[1] * nu : 0;
#pragma unroll
        for (int q = 0; q < W1R; ++q) {
            const int e = tid + q * nt, r = e / DQN_TILE;
            w1r[q] = e < n1 ? a.online[a.woff[1] + (int64_t)r * a.in[1] + u0 + (e - r * DQN_TILE)] : 0.0f;
        }
        if (a.code_w) {  // one thread per (row, cell): its six channels
            const uint16_t* R = reinterpret_cast<const uint16_t*>(Bt + DQN_TILE);  // [B][rw] words
            const int W = a.code_w, cells = W * W, cpg = lay::code_cpg(W), cpg8 = lay::code_cpg8(W);
            for (int e = tid; e < B * cells; e += nt) {
                const int b = e / cells, cl = e - b * cells;
                const int grp = (cl >= cpg) + (cl >= 2 * cpg) + (cl >= 3 * cpg);
                const uint32_t h = R[2 * b * rw + grp * cpg8 + (cl - grp * cpg)];
                const uint32_t obj = h & 7u, air = h >> 3;
                float* x = X + b * in4 + 6 * cl;
                x[0] = air ? 1.0f : 0.0f;
                x[1] = (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f;
                x[2] = obj == OBJ_DROPZONE ? 1.0f : 0.0f;
                x[3] = obj == OBJ_STATION ? 1.0f : 0.0f;
                x[4] = air ? (float)((int)(air & 0x7fu) - 1) / 100.0f : 0.0f;
                x[5] = obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f;
            }
            __syncthreads();
        }
        // the tile's pre-activations -> LDS Z [B][DQN_TILE] (after a code net's rows), then 16-B write-through
        dq_mm1(X, in4, Wt, xs0, 1, in, B, nu, [&](int b, int u, float z) { Z[b * DQN_TILE + u] = z + Bt[u]; });
#pragma unroll
        for (int q = 0; q < W1R; ++q) {
            const int e = tid + q * nt, r = e / DQN_TILE;
            if (e < n1) W1s[r * (DQN_TILE + 1) + (e - r * DQN_TILE)] = w1r[q];
        }
        __syncthreads();
        for (int e = tid; e < B * nu; e += nt) {  // the pre-activations as granules (the tails poll them)
            const int b = e / nu, u = e - b * nu;
            dq_granule_put(a.gz0 + ((int64_t)net * B + b) * out0 + u0 + u, epoch, Z[b * DQN_TILE + u]);
        }
        // hand-off: every wave drains its write-through stores, the workgroup barrier, one agent-scope ticket
        DQ_STAMP(3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(&a.ctr->arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // ---- 3. the weights: online workgroups their tile's layer-0 rows, target ones a share of the later
        // layers; the first DQN_PF per thread (weight, moments, target) are loaded into registers before the wait
        const bool later = net != 0;
        int64_t lo_i = 0, hi_i = (int64_t)nu * in;
        if (later) {
            const int64_t nw = a.wstart[L] - a.wstart[1], share = (nw + a.tiles0 - 1) / a.tiles0;
            lo_i = (int64_t)(w % a.tiles0) * share;
            hi_i = min(nw, lo_i + share);
        }
        const int64_t cnt = hi_i - lo_i;
        auto locate = [&](int64_t f, int& l, int& row, int& k) -> int64_t {  // element f -> (layer, row, k, index)
            if (!later) {
                const int u = (int)__umulhi((uint32_t)f, a.rm_in);
                l = 0;
                row = u0 + u;
                k = (int)f - u * in;
                return a.woff[0] + (int64_t)row * in + k;
            }
            const int64_t gi = a.wstart[1] + lo_i + f;
            l = 1;
            while (l + 1 < L && gi >= a.wstart[l + 1]) ++l;
            const int r0 = (int)(gi - a.wstart[l]), li = a.in[l];
            row = r0 / li;
            k = r0 - row * li;
            return a.woff[l] + r0;
        };
        float pp[DQN_PF], pm[DQN_PF], pv[DQN_PF], pt[DQN_PF];
        uint32_t px[DQN_PF];
#pragma unroll
        for (int q = 0; q < DQN_PF; ++q) {
            const int64_t f = tid + (int64_t)q * nt;
            pp[q] = pm[q] = pv[q] = pt[q] = 0.0f;
            px[q] = 0u;
            if (f < cnt) {
                int l, row, k;
                const int64_t wi = locate(f, l, row, k);
                pp[q] = a.online[wi];
                pm[q] = a.adam_m[wi];
                pv[q] = a.adam_v[wi];
                px[q] = a.pidx[wi];
                if (due) pt[q] = a.target[wi];
            }
        }
        // (online side, with a hidden layer) its units' layer-0 biases: moments and target loaded ahead too
        const bool b0up = net == 0 && L > 1 && tid < nu;
        float bm = 0.0f, bv = 0.0f, bt = 0.0f;
        if (b0up) {
            bm = a.adam_m[a.boff[0] + u0 + tid];
            bv = a.adam_v[a.boff[0] + u0 + tid];
            if (due) bt = a.target[a.boff[0] + u0 + tid];
        }
        // the online side (with a hidden layer) polls the layer-1 delta granules below instead of the epoch word
        const bool d1g = !later && L > 1;
        if (tid == 0) s_flag = d1g ? 1 : dq_wait(a, &a.ctr->pad[2], epoch);
        __syncthreads();
        DQ_STAMP(4);
        if (!s_flag) return;
        // the deltas (and the later layers' activations) the gradients read
        int* off = s_start;                                          // [2 (L - 1) + 1] prefix offsets
        const float** src = reinterpret_cast<const float**>(s_seg);  // [2 (L - 1)] sources
        float* Dz = Wt;   // [B][DQN_TILE] this tile's layer-0 deltas (the weight tile is dead)
        float* S = lds;   // later: D_l, H_{l-1} of every later layer (X is dead)
        if (!later && L == 1) {  // (no hidden layer: the output deltas are layer 0's)
            dq_stage(B * nu, [&](int i) { return dq_load_sc1(a.sd[0] + (i / nu) * out0 + u0 + i % nu); },
                     [&](int i, float d) { Dz[(i / nu) * DQN_TILE + i % nu] = d; });
        } else if (!later) {
            // this tile's layer-0 deltas from the handed-over layer-1 deltas: relu'(z0) * sum_j D1[b][j] W1[j][u]
            // (the oracle's backprop order over j), z0 still in Z
            const int o1 = a.out[1];
            for (int i = tid; i < B * o1; i += nt)  // the granules: polled in place (Guideline 16, R2)
                if (!dq_granule_get(a, a.gd1 + i, epoch, &D1s[i])) s_flag = 0;
            __syncthreads();
            if (!s_flag) return;
            DQ_STAMP(4);
            dq_mm1(D1s, o1, W1s, 1, DQN_TILE + 1, o1, B, nu, [&](int b, int u, float sum) {
                Dz[b * DQN_TILE + u] = Z[b * DQN_TILE + u] > 0.0f ? sum : 0.0f;
            });
        } else {
            if (tid == 0) {
                int ns = 0, tot = 0;
                for (int l = 1; l < L; ++l) {
                    off[ns] = tot;
                    src[ns++] = a.sd[l];
                    tot += B * a.out[l];
                    off[ns] = tot;
                    src[ns++] = a.sh[l - 1];
                    tot += B * a.in[l];
                }
                off[ns] = tot;
            }
            __syncthreads();
            dq_stage(off[2 * (L - 1)], [&](int i) {
                int g = 0;
                while (i >= off[g + 1]) ++g;
                return dq_load_sc1(src[g] + (i - off[g]));
            }, [&](int i, float v) { S[i] = v; });
        }
        __syncthreads();
        DQ_STAMP(6);
        // dW_l[row][k] = sum_b D_l[b][row] * H_{l-1}[b][k] in row order (layer 0: H = the sampled rows X)
        auto grad = [&](int l, int row, int k) {
            float g = 0.0f;
            if (!later) {
                for (int b = 0; b < B; ++b) g = g + Dz[b * DQN_TILE + (row - u0)] * X[b * in4 + k];
            } else {
                const int li = a.in[l], lo = a.out[l];
                const float* D = S + off[2 * (l - 1)];
                const float* H = S + off[2 * (l - 1) + 1];
                for (int b = 0; b < B; ++b) g = g + D[b * lo + row] * H[b * li + k];
            }
            return g;
        };
#pragma unroll
        for (int q = 0; q < DQN_PF; ++q) {
            const int64_t f = tid + (int64_t)q * nt;
            if (f < cnt) {
                int l, row, k;
                const int64_t wi = locate(f, l, row, k);
                float m = pm[q], v = pv[q];
                const float nwt = dq_adam(a, pp[q], grad(l, row, k), &m, &v, bc1, bc2);
                a.online[wi] = nwt;
                a.adam_m[wi] = m;
                a.adam_v[wi] = v;
#ifndef DRL_DIAG_NO_PACKW  // (diagnostic: timing without the packed image's writes; wrong results)
                qnet_pack_write_idx(a.pack, l, px[q], nwt);
#endif
                if (due) a.target[wi] = dq_blend(a, nwt, pt[q]);
            }
        }
        if (b0up) {  // (after the weights: the wave holding these threads is not held up) the layer-0 bias of unit u0 + tid: the batch sum of its deltas, Adam, packed, target blend
            const int u = tid;
            float g = 0.0f;
            for (int b = 0; b < B; ++b) g = g + Dz[b * DQN_TILE + u];
            const int64_t bi = a.boff[0] + u0 + u;
            const float nb = dq_adam(a, Bt[u], g, &bm, &bv, bc1, bc2);
            a.online[bi] = nb;
            a.adam_m[bi] = bm;
            a.adam_v[bi] = bv;
            a.pack.packed_b[a.pack.bias_off[0] + u0 + u] = nb;
            if (a.pack.code_w > 0)
                qnet_pack_write(a.pack, 0, qnet_pack_elem(0, u0 + u, -1, a.pack.kt[0], a.pack.code_w), -1, nb);
            if (due) a.target[bi] = dq_blend(a, nb, bt);
        }
        DQ_STAMP(7);
        for (int64_t base = tid + (int64_t)DQN_PF * nt; base < cnt; base += (int64_t)DQN_UB * nt) {  // (wide tiles)
            DqW ws[DQN_UB];
            int c = 0;
#pragma unroll
            for (int q = 0; q < DQN_UB; ++q) {
                const int64_t f = base + (int64_t)q * nt;
                if (f >= cnt) break;
                int l, row, k;
                const int64_t wi = locate(f, l, row, k);
                ws[q] = DqW{l, row, k, wi, grad(l, row, k)};
                c = q + 1;
            }
            if (c) dq_update_weights(a, ws, c, bc1, bc2, due);
        }
        DQ_STAMP(5);
        return;
    }

    // ---- 2. the tails: workgroup 0 the online net, 1 the target net
    if (flag != 0) return;
    const int n = blockIdx.x == 0 ? 0 : 1;
    const int mw = a.maxw;
    float* Pa = lds;                   // [B][mw] activations of the current layer
    float* Qa = lds + B * mw;          // [B][mw] the next layer's
    float* Ws = lds + 2 * B * mw;      // (no prefetch) one layer's weights, rows of in + 4 floats
    uint8_t* M = reinterpret_cast<uint8_t*>(Ws + (a.prefetch ? 0 : a.ws_floats));  // [L-1][B][mw] online ReLU masks
    const float* T = lds + a.region_a;  // the prefetched tail
    const int ns = a.ntail_of[n], g0 = n ? a.ntail_of[0] : 0;
    if (tid < ns) s_seg[tid] = a.tail[g0 + tid];
    if (tid <= ns) s_start[tid] = a.tail_start[g0 + tid] - a.tail_start[g0];
    __syncthreads();
    DQ_STAMP(1);
    const int ka = n == 0 ? a.ntail_a : ns, kb = n == 0 ? a.ntail_b : 0;  // (the online tail's parts A, B, C)
    dq_stage_segs(lds, s_seg, s_start, ka, s_tab);
    DQ_STAMP(7);
    // W_l^T for the backward pass: l >= 2 while the layer-0 workgroups run, W_1^T (only layer 0's deltas,
    // for its biases, read it) after the hand-off
    auto transpose = [&](int l) {
        const int li = a.in[l], lo = a.out[l];
        const float* W = T + a.tw[0][l];
        float* WT = lds + a.region_a + a.twt[l];
        for (int e = tid; e < lo * li; e += nt) {
            const int j = e / li, i = e - j * li;
            WT[i * (lo + 2) + j] = W[j * (li + 2) + i];
        }
    };
    if (n == 0 && a.prefetch) {
        __syncthreads();
        for (int l = 2; l < L; ++l) transpose(l);
    }
    DQ_STAMP(2);
    if (tid == 0) s_flag = 1;
    __syncthreads();
    DQ_STAMP(3);
    Pa = dq_forward(a, n, Pa, Qa, Ws, M, T, epoch, &s_flag);
    if (!Pa) return;
    Qa = Pa == lds ? lds + B * mw : lds;
    DQ_STAMP(4);
    const int A = a.out[L - 1];
    if (n == 1) {  // max_a Q_target, handed over as granules
        for (int b = tid; b < B; b += nt) {
            float mx = Pa[b * mw];
            for (int j = 1; j < A; ++j) mx = Pa[b * mw + j] > mx ? Pa[b * mw + j] : mx;  // jnp.max
            dq_granule_put(a.gmx + b, epoch, mx);
        }
        return;
    }
    for (int b = tid; b < B; b += nt)
        for (int j = 0; j < A; ++j) s_q[b * 8 + j] = Pa[b * mw + j];
    dq_stage_segs(lds, s_seg + ka, s_start + ka, kb, s_tab);  // B: the rows' action, reward, done
    for (int b = tid; b < B; b += nt)
        if (!dq_granule_get(a, a.gmx + b, epoch, &s_mx[b])) s_flag = 0;
    __syncthreads();
    if (!s_flag) return;
    DQ_STAMP(5);
    float loss = 0.0f;
    for (int b = tid; b < B; b += nt) {
        const int act = __float_as_int(T[a.tr + b]);
        const float rew = T[a.tr + B + b];
        const float notdone = T[a.tr + 2 * B + b] != 0.0f ? 0.0f : 1.0f;
        const float td = rew + (a.gamma * s_mx[b]) * notdone;
        const bool ok = act >= 0 && act < A;
        s_d[b] = (ok ? s_q[b * 8 + act] : td) - td;  // (an action outside [0, A) adds nothing)
        s_act[b] = ok ? act : -1;
    }
    __syncthreads();
    for (int b = 0; b < B; ++b) loss = loss + s_d[b] * s_d[b];
    loss = loss / (float)B;  // jnp.mean(jnp.square(q - td))
    // d loss / d q[b][a_b] = 2 (q - td) / B: the output layer's deltas
    float* D = Pa;   // [B][mw] deltas of layer l
    float* D2 = Qa;  // [B][mw] deltas of layer l - 1
    for (int o = tid; o < B * A; o += nt) {
        const int b = o / A, j = o - b * A;
        const float dq = (s_act[b] == j) ? (s_d[b] + s_d[b]) / (float)B : 0.0f;
        D[b * mw + j] = dq;
        dq_store_sc1(a.sd[L - 1] + o, dq);
        if (L == 2) dq_granule_put(a.gd1 + o, epoch, dq);  // (layer 1's deltas: the online layer-0 workgroups)
    }
    __syncthreads();
    // each layer's bias gradient, the batch sum of its deltas in row order, as its deltas appear (the bias
    // updates run behind the hand-off; layer 0's: the online layer-0 workgroups, which form its deltas)
    auto bias_grad = [&](int l, const float* Dl) {
        for (int j = tid; j < a.out[l]; j += nt) {
            float g = 0.0f;
            for (int b = 0; b < B; ++b) g = g + Dl[b * mw + j];
            s_gb[l][j] = g;
        }
    };
    bias_grad(L - 1, D);
    // delta_{l-1}[b][i] = relu'(z) * sum_j D[b][j] W[j][i] (the same micro-tiles over the out index j;
    // prefetched: on W_l^T, rows of lo + 2 floats, the forward's bank pattern), published to sd[l - 1]
    auto backward = [&](int l) {
        const int lo = a.out[l], li = a.out[l - 1], ls = li + 4;
        if (!a.prefetch && l < L - 1) {  // (W_{L-1} is still staged from the forward pass)
            __syncthreads();
            dq_stage_w(a, a.online, l, Ws);  // (this step's weights: the update workgroups write them after)
            __syncthreads();
        }
        if (a.prefetch)
            dq_mm(D, mw, 1, T + a.twt[l], lo + 2, 1, lo, B, li, [&](int b, int i, float s) { D2[b * mw + i] = s; });
        else
            dq_mm(D, mw, 1, Ws, 1, ls, lo, B, li, [&](int b, int i, float s) { D2[b * mw + i] = s; });
        __syncthreads();
        for (int e = tid; e < B * li; e += nt) {  // relu'(z): the online forward's masks
            const int b = e / li, i = e - b * li;
            if (!M[((l - 1) * B + b) * mw + i]) D2[b * mw + i] = 0.0f;
        }
        __syncthreads();
        DQ_STAMP(12 + L - 1 - l);
        if (l == 2)  // layer 1's deltas, also as granules: the online layer-0 workgroups poll them
            for (int e = tid; e < B * li; e += nt) {
                const int b = e / li, i = e - b * li;
                dq_granule_put(a.gd1 + e, epoch, D2[b * mw + i]);
            }
        dq_publish(D2, mw, a.sd[l - 1], li, B, li);
        bias_grad(l - 1, D2);
        float* t = D;
        D = D2;
        D2 = t;
    };
    // down to layer 1's deltas before the hand-off: the online layer-0 workgroups form their own layer-0
    // deltas from them (3. above)
    for (int l = L - 1; l >= 2; --l) backward(l);
    DQ_STAMP(15);
    // hand the deltas and activations over: every wave drains, the barrier, the epoch word
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && !a.drop_handoff)
        __hip_atomic_store((gu32*)&a.ctr->pad[2], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    DQ_STAMP(6);
#ifdef DRL_DQN_STAMPS
    if (threadIdx.x == 0) {
        a.stamps[1002] = clock64();
        a.stamps[1003] = wall_clock64();
    }
#endif
    dq_stage_segs(lds, s_seg + ka + kb, s_start + ka + kb, ns - ka - kb, s_tab);  // C: for the bias updates
    __syncthreads();
    // the biases of layers >= 1 (layer 0's too without a hidden layer): Adam on the gradients formed above,
    // the packed image, the target blend
    for (int l = L > 1 ? 1 : 0; l < L; ++l) {
        const int lo = a.out[l];
        for (int j = tid; j < lo; j += nt) {
            const float g = s_gb[l][j];
            const int64_t bi = a.boff[l] + j;
            float m = T[a.tm[l] + j], v = T[a.tv[l] + j];
            const float b0 = T[a.tb[0][l] + j], tb = T[a.tb[1][l] + j];
            const float nb = dq_adam(a, b0, g, &m, &v, bc1, bc2);
            a.online[bi] = nb;
            a.adam_m[bi] = m;
            a.adam_v[bi] = v;
            a.pack.packed_b[a.pack.bias_off[l] + j] = nb;
            if (l == 0 && a.pack.code_w > 0)
                qnet_pack_write(a.pack, 0, qnet_pack_elem(0, j, -1, a.pack.kt[0], a.pack.code_w), -1, nb);
            if (due) a.target[bi] = dq_blend(a, nb, tb);
        }
    }
    DQ_STAMP(14);
    if (tid == 0) {  // every layer-0 workgroup has read this step's counters (its ticket): then write them
        s_flag = dq_wait(a, &a.ctr->arrive, (uint32_t)a.nblk0);
        __hip_atomic_store((gu32*)&a.ctr->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_flag) dq_finish(a, ctr, 1, loss, bc1, bc2);
}

// The replay slots the next drl_dqn_train launch samples (its step counter as it stands on the stream):
// the same dq_sample draws, for a caller that gathers those rows first (the sharded global learner)
__global__ void drl_dqn_sample_kernel(const DqnCounters* c, uint64_t seed, int batch, int64_t size, int64_t* out) {
    const int b = threadIdx.x;
    if (b < batch) out[b] = dq_sample(seed, c->step, b, size);
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

hipError_t launch_dqn_train(const LearnArgs& a, size_t lds, hipStream_t s) {
    if (a.trained)
        hipLaunchKernelGGL(drl_dqn_train_kernel<true>, dim3((unsigned)a.nblk0 + 2), dim3(DQN_THREADS), lds, s, a);
    else
        hipLaunchKernelGGL(drl_dqn_train_kernel<false>, dim3(1), dim3(DQN_THREADS), 0, s, a);
    return hipGetLastError();
}

int dqn_train_resident_capacity(size_t lds, int num_cus) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, drl_dqn_train_kernel<true>, DQN_THREADS, lds) != hipSuccess)
        return -1;
    return per_cu * num_cus;
}

hipError_t launch_dqn_sample(const void* counters, uint64_t seed, int batch, int64_t size, int64_t* out, hipStream_t s) {
    hipLaunchKernelGGL(drl_dqn_sample_kernel, dim3(1), dim3(64), 0, s, static_cast<const DqnCounters*>(counters), seed,
                       batch, size, out);
    return hipGetLastError();
}

hipError_t launch_dqn_init(void* counters, float epsilon, hipStream_t s) {
    hipLaunchKernelGGL(drl_dqn_init_kernel, dim3(1), dim3(64), 0, s, static_cast<DqnCounters*>(counters), epsilon);
    return hipGetLastError();
}

}  // namespace drl
