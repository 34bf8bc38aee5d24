// dronerl_qnet.hip — the on-device DQN consumer of the observation (SURVEY.md
// §8 F1): dense Q-network forward + epsilon-greedy act for every env, and the
// replay buffer's add_many.
//
// Reference: jax_impl/agents/dqn.py DenseQNetwork (:47-63: Dense(h) + relu per
// hidden layer, Dense(5)), DQNAgent.act (:132-146: uniform < epsilon ? random
// action : argmax Q), train_jax.py:42-49 (drone 0 of every env follows the
// agent), jax_impl/buffers.py:57-80 ReplayBuffer.add_many.
//
// MFMA layout (gfx950 v_mfma_f32_16x16x32_bf16, bf16 operands, f32
// accumulate): envs are the MFMA column dimension, so layer l computes
// H_lᵀ = W_l · H_{l-1}ᵀ in 16(units) x 16(envs) tiles over 32-wide K-slices.
// Lane l (c = l&15, g = l>>4) holds A[row c][k(g, j)] and B[k(g, j)][col c]
// for j = 0..7, and the accumulator holds rows 4g + i of column c in register
// i.  With the K order k(g, j) = j<4 ? 4g+j : 16+4g+(j-4), registers 0..3 of
// accumulator tiles 2s and 2s+1 are exactly the B fragment of the next
// layer's K-slice s (activations never leave registers), and for the input
// layer the four lanes of an env read 64 contiguous bytes of its row per load.
// Weights are packed once (drl_qnet_pack) into that lane-fragment order and
// staged into LDS per workgroup (one 16-B ds_read per lane per MFMA).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dronerl_internal.h"

namespace drl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t qn_splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// The exploration rate: the argument, or the learner's device counter
// (drl_qnet_act_eps).
__device__ __forceinline__ float qn_eps(const QnetArgs& a) { return a.eps_ptr ? *a.eps_ptr : a.epsilon; }

// K index within a 32-wide slice of fragment element j for lane group g (see
// the header comment).
__device__ __forceinline__ int frag_k(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

// ------------------------------------------------------------------ pack ---
// One thread per packed bf16 element: fragment (m, t) of layer l is 64 lanes x
// 8 elements, element j of lane (c, g) = W_l[16m + c][32t + frag_k(g, j)]
// (torch nn.Linear layout [out][in]); zero outside the matrix.  Biases follow
// as f32.
__global__ void drl_qnet_pack_kernel(QnetPack p) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < p.n_wfrag_elems) {
        int l = 0;
        while (l + 1 < p.n_layers && i >= (int64_t)p.frag_src[l + 1] * 8) ++l;
        const int64_t e = i - (int64_t)p.frag_src[l] * 8;  // element within the layer
        // (a code net: layer 0 in the policy code's K order, its bias in the
        // first padding slot of lane group 0 -- qnet_pack_slot)
        const PackSlot s = qnet_pack_slot(l, e, p.kt[l], p.code_w, p.in[l]);
        float w = (s.row < p.out[l] && s.k >= 0 && s.k < p.in[l]) ? p.w[l][(int64_t)s.row * p.in[l] + s.k] : 0.0f;
        if (s.k < 0) w = s.row < p.out[l] ? p.b[l][s.row] : 0.0f;
        // (the charge channel's 1/100 moves into its weights: the kernel feeds
        // the integer charge, exact in fp16, so no input needs an x_lo product)
        qnet_pack_write(p, l, e, s.k, w);
    } else if (i < p.n_wfrag_elems + p.n_bias) {
        const int64_t bi = i - p.n_wfrag_elems;
        int l = 0;
        while (l + 1 < p.n_layers && bi >= p.bias_off[l + 1]) ++l;
        const int u = (int)(bi - p.bias_off[l]);
        p.packed_b[bi] = u < p.out[l] ? p.b[l][u] : 0.0f;
    }
}

// ------------------------------------------------------------------- act ---
// One workgroup of QN_WAVES waves per CU: the packed net (99 KB for the C3
// net) is staged into LDS once per workgroup, and each wave runs 16-env
// tiles.  Input K-slices stream from HBM into a ring of QN_RING register
// buffers that rolls across tile boundaries: a buffer is re-issued for the
// slice QN_RING positions ahead as soon as it is consumed.  The slice count is
// padded to a multiple of QN_RING (zero weight fragments), so ring positions
// are static and the loads need no masks or branches.
constexpr int QN_WAVES = lay::qn_waves;
constexpr int QN_MAXT = 8;    // 16-unit tiles per hidden layer (hidden <= 128)
constexpr int QN_RING = lay::qn_ring;  // K-slices in flight per wave
constexpr int QN_TILES = lay::qn_tiles;  // env tiles per pass sharing each weight fragment
#ifndef DRL_QN_TILES_F32
#define DRL_QN_TILES_F32 1
#endif
constexpr int QN_TILES_F32 = DRL_QN_TILES_F32;  // the same for DRL_QNET_F32 (two accumulator sets)

__device__ __forceinline__ bf16x8 lds_frag(const uint4* base, int frag, int lane) {
    const uint4 v = base[frag * 64 + lane];
    bf16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// TP env tiles per pass share every weight fragment read from LDS (TP MFMAs per
// fragment): a wave's pass covers TP*16 envs.
template <int NT0>
__global__ void __launch_bounds__(64 * QN_WAVES) drl_qnet_act_kernel(QnetArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 15, g = lane >> 4;
    constexpr int nt0 = NT0;  // first-layer tiles (compile time: no branches around its MFMAs)
    constexpr int TP = QN_TILES;
    const int64_t ntiles = (a.E + 15) / 16;
    const int64_t ngroups = (ntiles + TP - 1) / TP;
    const int64_t gstride = (int64_t)gridDim.x * QN_WAVES;
    const int KP = a.kt0;                 // padded to a multiple of QN_RING
    const int rounds = KP / QN_RING;
    float raw[TP][QN_RING][8];
    // slice t (features 32t + frag_k(g, 0..7)) of the env row at byte offset
    // `rowb` from obs: two 16-B loads; the four lanes of the env cover 64
    // contiguous bytes per load (rows are 8-B aligned at 294 floats: gfx950
    // serves 8-B aligned dwordx4, tools/unaligned_probe.hip).  A quad past
    // in_features reads the row's last quad (zero weights there); the quad that
    // straddles in_features (in_features % 4 == 2) takes its valid pair from
    // the upper half of that last quad.
    const char* obase = reinterpret_cast<const char*>(a.obs);
    auto load_slice = [&](uint32_t rowb, int t, float (&dst)[8]) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ks = 32 * t + 16 * q + 4 * g;
            const uint32_t off = rowb + 4u * (uint32_t)min(ks, a.in_features - 4);
            float4 v;
            __builtin_memcpy(&v, __builtin_assume_aligned(obase + off, 8), 16);
            const bool straddle = ks == a.in_features - 2;
            dst[4 * q + 0] = straddle ? v.z : v.x;
            dst[4 * q + 1] = straddle ? v.w : v.y;
            dst[4 * q + 2] = v.z;
            dst[4 * q + 3] = v.w;
        }
    };
    auto row_of = [&](int64_t t) {
        const int64_t env = t * 16 + c;
        return (uint32_t)((env < a.E ? env : a.E - 1) * a.obs_stride * 4);
    };
    const int64_t grp0 = (int64_t)blockIdx.x * QN_WAVES + wave;
    int64_t grp = grp0;
    uint32_t row[TP];
#pragma unroll
    for (int h = 0; h < TP; ++h) row[h] = row_of(TP * (grp < ngroups ? grp : 0) + h);
    // ---- the first ring of slices, then the packed net by LDS-DMA (no
    // registers; every 16-B piece in flight at once)
#pragma unroll
    for (int i = 0; i < QN_RING; ++i)
#pragma unroll
        for (int h = 0; h < TP; ++h) load_slice(row[h], i, raw[h][i]);
    for (int v0 = wave * 64; v0 < a.lds_vec; v0 += 64 * QN_WAVES)
        if (v0 + lane < a.lds_vec)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.packed + v0 + lane),
                                             (__attribute__((address_space(3))) void*)(wl + v0), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* bias = reinterpret_cast<const float*>(wl + a.frag_total);
    const uint4* W0 = wl + a.frag_off[0];

    for (; grp < ngroups; grp += gstride) {
        const int64_t ngrp = grp + gstride;
        uint32_t nrow[TP];
#pragma unroll
        for (int h = 0; h < TP; ++h) nrow[h] = row_of(TP * (ngrp < ngroups ? ngrp : grp) + h);
        f32x4 acc[TP][QN_MAXT];
#pragma unroll
        for (int h = 0; h < TP; ++h)
#pragma unroll
            for (int m = 0; m < QN_MAXT; ++m) acc[h][m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        // ---- layer 0 over the ring.  Refill mode per round (compile time):
        // 0 = slice t + RING of this group (all rounds but the last), 1 = of
        // the next group, 2 = none (this wave's last group)
        auto round = [&](int rd, auto mode) {
            constexpr int MODE = decltype(mode)::value;
#pragma unroll
            for (int i = 0; i < QN_RING; ++i) {
                const int t = rd * QN_RING + i;
                bf16x8 b[TP];
#pragma unroll
                for (int h = 0; h < TP; ++h) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) b[h][j] = (__bf16)raw[h][i][j];
                    if constexpr (MODE == 0) load_slice(row[h], t + QN_RING, raw[h][i]);
                    else if constexpr (MODE == 1) load_slice(nrow[h], t + QN_RING - KP, raw[h][i]);
                }
#pragma unroll
                for (int m = 0; m < nt0; ++m) {
                    const bf16x8 w = lds_frag(W0, m * KP + t, lane);
#pragma unroll
                    for (int h = 0; h < TP; ++h) acc[h][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, b[h], acc[h][m], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);  // A reads next to their MFMAs (register pressure)
            }
        };
        for (int rd = 0; rd + 1 < rounds; ++rd) round(rd, std::integral_constant<int, 0>{});
        if (ngrp < ngroups) round(rounds - 1, std::integral_constant<int, 1>{});
        else round(rounds - 1, std::integral_constant<int, 2>{});
#pragma unroll
        for (int h = 0; h < TP; ++h) row[h] = nrow[h];
        // ---- hidden layers 1..n_hidden-1 and the output layer: B operands in registers
        int nt_prev = nt0;
        const float* bprev = bias + a.bias_off[0];
        for (int l = 1; l <= a.n_hidden; ++l) {
            // activation (bias + ReLU) of the previous layer as bf16 B fragments:
            // K-slice s = registers of tiles 2s (j < 4) and 2s + 1 (j >= 4)
            bf16x8 bf[TP][QN_MAXT / 2];
#pragma unroll
            for (int h = 0; h < TP; ++h) {
#pragma unroll
                for (int s2 = 0; s2 < QN_MAXT / 2; ++s2) {
                    if (2 * s2 < nt_prev) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int m = 2 * s2 + (j >> 2), i = j & 3;
                            bf[h][s2][j] = (__bf16)fmaxf(acc[h][m][i] + bprev[16 * m + 4 * g + i], 0.0f);
                        }
                    }
                }
            }
            const int nt_l = (l < a.n_hidden) ? a.nt[l] : 1;  // output layer: one tile (<= 16 actions)
            const int kt = nt_prev / 2;
#pragma unroll
            for (int h = 0; h < TP; ++h)
#pragma unroll
                for (int m = 0; m < QN_MAXT; ++m) acc[h][m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            const uint4* Wl = wl + a.frag_off[l];
#pragma unroll
            for (int t = 0; t < QN_MAXT / 2; ++t) {
                if (t < kt) {
#pragma unroll
                    for (int m = 0; m < QN_MAXT; ++m) {
                        if (m < nt_l) {
                            const bf16x8 w = lds_frag(Wl, m * kt + t, lane);
#pragma unroll
                            for (int h = 0; h < TP; ++h)
                                acc[h][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, bf[h][t], acc[h][m], 0, 0, 0);
                        }
                    }
                }
            }
            nt_prev = nt_l;
            bprev = bias + a.bias_off[l];
        }
        // ---- Q values: actions 0..3 in registers 0..3 of the g = 0 lanes,
        // 4..7 in those of the g = 1 lanes (column = env)
#pragma unroll
        for (int h = 0; h < TP; ++h) {
            float q[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float own = acc[h][0][i] + bprev[4 * g + i];
                const float hi = __shfl(own, c + 16);  // g = 1 lane of this env
                q[i] = own;
                q[i + 4] = hi;
            }
            const int64_t env = (TP * grp + h) * 16 + c;
            if (g == 0 && env < a.E) {
                int best = 0;  // jnp.argmax: first maximum
                for (int i = 1; i < a.n_actions; ++i) best = q[i] > q[best] ? i : best;
                const uint64_t ge = (uint64_t)(a.env_offset + env);
                const uint64_t hsh = qn_splitmix64(a.seed ^ qn_splitmix64((a.step << 40) ^ (ge << 8) ^ 0xa5ull));
                const float u = (float)(hsh >> 40) * (1.0f / 16777216.0f);
                const int rnd = (int)(((hsh & 0xffffffffull) * (uint64_t)a.n_actions) >> 32);
                a.actions[env * a.action_stride] = (u < qn_eps(a)) ? rnd : best;
                if (a.q)
                    for (int i = 0; i < a.n_actions; ++i) a.q[env * a.n_actions + i] = q[i];
            }
        }
    }
    if (a.synth_n > 1) {
        // drl_synth_actions' columns 1..N-1 of this wave's envs, last: stores
        // issued before the net's LDS-DMA wait (vmcnt counts them) would delay
        // the first group
        const uint32_t nd = (uint32_t)a.synth_n - 1u;
        const uint32_t per = (uint32_t)(TP * 16) * nd;
        for (int64_t gg = grp0; gg < ngroups; gg += gstride) {
            for (uint32_t k = (uint32_t)lane; k < per; k += 64u) {
                const uint32_t el = k / nd;
                const int64_t env = TP * 16 * gg + el;
                const uint64_t drone = 1u + (k - el * nd);
                if (env < a.E) {
                    const uint64_t ctr = (a.synth_step << 40) ^ ((uint64_t)(a.env_offset + env) << 8) ^ drone;
                    const uint64_t h = qn_splitmix64(a.synth_seed ^ qn_splitmix64(ctr));
                    a.actions[env * a.action_stride + (int64_t)drone] = (int32_t)(((h >> 32) * 5ull) >> 32);
                }
            }
        }
    }
}

// ---------------------------------------------------------- act, F32 ---
// DRL_QNET_F32: the same dataflow with every operand v split into fp16
// hi = fp16(v) and lo = fp16((v - hi) * 2^11) (exact up to 2^-23 |v|).
// Per tile and K-slice three v_mfma_f32_16x16x32_f16: acc += Whi*xhi and
// acl += Wlo*xhi + Whi*xlo; a layer's value is acc + 2^-11 * acl (+ bias).
// bf16 products would need three pieces per operand (six MFMAs); fp16's
// 11-bit significand needs two.  The hi fragments sit where the bf16 ones do
// (LDS), the later layers' lo fragments after the biases (LDS); layer 0's lo
// fragments stay in global memory (L2-resident, 1 KB per fragment) because
// both sets of the 294->128 layer do not fit 160 KB of LDS.  A slice's lo
// fragments are loaded at its start and used after its hi products.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f16x8 as_f16x8(const uint4 v) {
    f16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// `bad` collects operands outside fp16's range (|v| >= 65520 rounds hi to
// inf; NaN stays NaN): the split would turn them into NaN Q values, so the
// kernel flags DRL_ERR_QNET_RANGE instead of failing silently.
// Weights (and a code net's layer-0 bias) are range-checked when packed (the
// pack status word, read at the end of every f32 act).  With finite fp16
// operands below 65520 and K <= 512, an f32 pre-activation is finite, so the
// ReLU's fmaxf never sees a NaN that these two checks did not flag.
__device__ __forceinline__ void split_f16(const float (&v)[8], f16x8& hi, f16x8& lo, bool& bad) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)v[j];
        hi[j] = h;
        lo[j] = (_Float16)((v[j] - (float)h) * 2048.0f);
        bad |= !(__builtin_fabsf(v[j]) < 65520.0f);
    }
}

#define MFMA_F16 __builtin_amdgcn_mfma_f32_16x16x32_f16

// LO0 (the layout whenever layer 0's two fragment sets fit, as at 294->128):
// layer 0's hi and lo fragments are the LDS image and the later layers'
// fragments and the biases are read from global memory (L2) instead, which
// moves a tile's L2 weight reads from 80 KB (layer 0's lo set) to the later
// layers' few KB.
template <int NT0, int TP, bool LO0>
__global__ void __launch_bounds__(64 * QN_WAVES) drl_qnet_act_f32_kernel(QnetArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 15, g = lane >> 4;
    constexpr int nt0 = NT0;
    const int64_t ntiles = (a.E + 15) / 16;
    const int64_t ngroups = (ntiles + TP - 1) / TP;
    const int64_t gstride = (int64_t)gridDim.x * QN_WAVES;
    const int KP = a.kt0;
    const int rounds = KP / QN_RING;
    constexpr float kLo = 1.0f / 2048.0f;
    float raw[TP][QN_RING][8];
    // the observation rows by buffer loads (32-bit offsets; the host checks obs < 4 GiB)
    const auto obuf = __builtin_amdgcn_make_buffer_rsrc((void*)a.obs, 0, (int)(a.E * a.obs_stride * 4), 0x00020000);
    auto load_slice = [&](uint32_t rowb, int t, float (&dst)[8]) {  // as in drl_qnet_act_kernel
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ks = 32 * t + 16 * q + 4 * g;
            const uint32_t off = rowb + 4u * (uint32_t)min(ks, a.in_features - 4);
            const auto raw4 = __builtin_amdgcn_raw_buffer_load_b128(obuf, (int)off, 0, 0);
            float4 v;
            __builtin_memcpy(&v, &raw4, 16);
            const bool straddle = ks == a.in_features - 2;
            dst[4 * q + 0] = straddle ? v.z : v.x;
            dst[4 * q + 1] = straddle ? v.w : v.y;
            dst[4 * q + 2] = v.z;
            dst[4 * q + 3] = v.w;
        }
    };
    auto row_of = [&](int64_t t) {
        const int64_t env = t * 16 + c;
        return (uint32_t)((env < a.E ? env : a.E - 1) * a.obs_stride * 4);
    };
    const int64_t grp0 = (int64_t)blockIdx.x * QN_WAVES + wave;
    int64_t grp = grp0;
    uint32_t row[TP];
#pragma unroll
    for (int h = 0; h < TP; ++h) row[h] = row_of(TP * (grp < ngroups ? grp : 0) + h);
    // layer-0 lo fragments (global, L2-resident): buffer loads with the lane's
    // 16-B offset in one VGPR and the fragment offset in an SGPR
    const auto glo0 = __builtin_amdgcn_make_buffer_rsrc((void*)(a.packed + (LO0 ? 0 : a.frag_lo_off[0])), 0,
                                                         nt0 * KP * 1024, 0x00020000);
#pragma unroll
    for (int i = 0; i < QN_RING; ++i)
#pragma unroll
        for (int h = 0; h < TP; ++h) load_slice(row[h], i, raw[h][i]);
    for (int v0 = wave * 64; v0 < a.lds_vec; v0 += 64 * QN_WAVES)
        if (v0 + lane < a.lds_vec)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.packed + v0 + lane),
                                             (__attribute__((address_space(3))) void*)(wl + v0), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool bad = false;  // an operand outside fp16's range (split_f16)
    const float* bias = LO0 ? reinterpret_cast<const float*>(a.packed + a.bias_vec)
                            : reinterpret_cast<const float*>(wl + a.frag_total);
    const uint4* W0 = wl + a.frag_off[0];
    const uint4* W0lo = wl + (LO0 ? a.frag_lo_off[0] : 0);
    const uint4* Wsrc = LO0 ? a.packed : wl;  // the later layers' fragments

    for (; grp < ngroups; grp += gstride) {
        const int64_t ngrp = grp + gstride;
        uint32_t nrow[TP];
#pragma unroll
        for (int h = 0; h < TP; ++h) nrow[h] = row_of(TP * (ngrp < ngroups ? ngrp : grp) + h);
        f32x4 acc[TP][QN_MAXT], acl[TP][QN_MAXT];
#pragma unroll
        for (int h = 0; h < TP; ++h)
#pragma unroll
            for (int m = 0; m < QN_MAXT; ++m) acc[h][m] = acl[h][m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        auto round = [&](int rd, auto mode) {
            constexpr int MODE = decltype(mode)::value;
#pragma unroll
            for (int i = 0; i < QN_RING; ++i) {
                const int t = rd * QN_RING + i;
                uint4 wlo[NT0];  // the slice's lo fragments (L2), used after the hi products
                if constexpr (!LO0) {
#pragma unroll
                    for (int m = 0; m < nt0; ++m) {
                        const auto v = __builtin_amdgcn_raw_buffer_load_b128(glo0, lane * 16, (m * KP + t) * 1024, 0);
                        __builtin_memcpy(&wlo[m], &v, 16);
                    }
                }
                f16x8 bh[TP], bl[TP];
#pragma unroll
                for (int h = 0; h < TP; ++h) {
                    split_f16(raw[h][i], bh[h], bl[h], bad);
                    if constexpr (MODE == 0) load_slice(row[h], t + QN_RING, raw[h][i]);
                    else if constexpr (MODE == 1) load_slice(nrow[h], t + QN_RING - KP, raw[h][i]);
                }
#pragma unroll
                for (int m = 0; m < nt0; ++m) {
                    const f16x8 wh = as_f16x8(W0[(m * KP + t) * 64 + lane]);
#pragma unroll
                    for (int h = 0; h < TP; ++h) {
                        acc[h][m] = MFMA_F16(wh, bh[h], acc[h][m], 0, 0, 0);
                        acl[h][m] = MFMA_F16(wh, bl[h], acl[h][m], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int m = 0; m < nt0; ++m) {
                    const f16x8 wo = as_f16x8(LO0 ? W0lo[(m * KP + t) * 64 + lane] : wlo[m]);
#pragma unroll
                    for (int h = 0; h < TP; ++h) acl[h][m] = MFMA_F16(wo, bh[h], acl[h][m], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        for (int rd = 0; rd + 1 < rounds; ++rd) round(rd, std::integral_constant<int, 0>{});
        if (ngrp < ngroups) round(rounds - 1, std::integral_constant<int, 1>{});
        else round(rounds - 1, std::integral_constant<int, 2>{});
#pragma unroll
        for (int h = 0; h < TP; ++h) row[h] = nrow[h];
        int nt_prev = nt0;
        const float* bprev = bias + a.bias_off[0];
        for (int l = 1; l <= a.n_hidden; ++l) {
            f16x8 ah[TP][QN_MAXT / 2], al[TP][QN_MAXT / 2];
#pragma unroll
            for (int h = 0; h < TP; ++h) {
#pragma unroll
                for (int s2 = 0; s2 < QN_MAXT / 2; ++s2) {
                    if (2 * s2 < nt_prev) {
                        float v[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int m = 2 * s2 + (j >> 2), i = j & 3;
                            v[j] = fmaxf((acc[h][m][i] + acl[h][m][i] * kLo) + bprev[16 * m + 4 * g + i], 0.0f);
                        }
                        split_f16(v, ah[h][s2], al[h][s2], bad);
                    }
                }
            }
            const int nt_l = (l < a.n_hidden) ? a.nt[l] : 1;
            const int kt = nt_prev / 2;
#pragma unroll
            for (int h = 0; h < TP; ++h)
#pragma unroll
                for (int m = 0; m < QN_MAXT; ++m) acc[h][m] = acl[h][m] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            const uint4* Wl = Wsrc + a.frag_off[l];
            const uint4* Wlo = Wsrc + a.frag_lo_off[l];
#pragma unroll
            for (int t = 0; t < QN_MAXT / 2; ++t) {
                if (t < kt) {
#pragma unroll
                    for (int m = 0; m < QN_MAXT; ++m) {
                        if (m < nt_l) {
                            const f16x8 wh = as_f16x8(Wl[(m * kt + t) * 64 + lane]);
                            const f16x8 wo = as_f16x8(Wlo[(m * kt + t) * 64 + lane]);
#pragma unroll
                            for (int h = 0; h < TP; ++h) {
                                acc[h][m] = MFMA_F16(wh, ah[h][t], acc[h][m], 0, 0, 0);
                                acl[h][m] = MFMA_F16(wh, al[h][t], acl[h][m], 0, 0, 0);
                                acl[h][m] = MFMA_F16(wo, ah[h][t], acl[h][m], 0, 0, 0);
                            }
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // fragment reads next to their MFMAs (register pressure)
            }
            nt_prev = nt_l;
            bprev = bias + a.bias_off[l];
        }
#pragma unroll
        for (int h = 0; h < TP; ++h) {
            float q[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float own = (acc[h][0][i] + acl[h][0][i] * kLo) + bprev[4 * g + i];
                const float hi = __shfl(own, c + 16);
                q[i] = own;
                q[i + 4] = hi;
            }
            const int64_t env = (TP * grp + h) * 16 + c;
            if (g == 0 && env < a.E) {
                int best = 0;
                for (int i = 1; i < a.n_actions; ++i) best = q[i] > q[best] ? i : best;
                const uint64_t ge = (uint64_t)(a.env_offset + env);
                const uint64_t hsh = qn_splitmix64(a.seed ^ qn_splitmix64((a.step << 40) ^ (ge << 8) ^ 0xa5ull));
                const float u = (float)(hsh >> 40) * (1.0f / 16777216.0f);
                const int rnd = (int)(((hsh & 0xffffffffull) * (uint64_t)a.n_actions) >> 32);
                a.actions[env * a.action_stride] = (u < qn_eps(a)) ? rnd : best;
                if (a.q)
                    for (int i = 0; i < a.n_actions; ++i) a.q[env * a.n_actions + i] = q[i];
            }
        }
    }
    bad |= lane == 0 && reinterpret_cast<const int32_t*>(a.packed + a.status_vec)[0] != 0;  // pack range flag
    if (__ballot(bad) && lane == 0 && a.err) atomicOr(a.err, DRL_ERR_QNET_RANGE);
    if (a.synth_n > 1) {  // as in drl_qnet_act_kernel
        const uint32_t nd = (uint32_t)a.synth_n - 1u;
        const uint32_t per = (uint32_t)(TP * 16) * nd;
        for (int64_t gg = grp0; gg < ngroups; gg += gstride) {
            for (uint32_t k = (uint32_t)lane; k < per; k += 64u) {
                const uint32_t el = k / nd;
                const int64_t env = TP * 16 * gg + el;
                const uint64_t drone = 1u + (k - el * nd);
                if (env < a.E) {
                    const uint64_t ctr = (a.synth_step << 40) ^ ((uint64_t)(a.env_offset + env) << 8) ^ drone;
                    const uint64_t h = qn_splitmix64(a.synth_seed ^ qn_splitmix64(ctr));
                    a.actions[env * a.action_stride + (int64_t)drone] = (int32_t)(((h >> 32) * 5ull) >> 32);
                }
            }
        }
    }
}

// ----------------------------------------------------- act from the code ---
// drl_qnet_act_code: the f32 act with its input built from the policy code
// the step wrote (write_obs_wave<CODE>: drone 0's window, one u16 per cell, 128 B
// per env at radius 3) instead of read from the f32 observation (1,176 B per
// env, 8-B-aligned rows read as strided 128-B slices): the input of a 16-env
// tile is 2 KB, contiguous, and the kernel is no longer bound by the latency
// of observation reads (C3: 77 MB per step).  The channels are computed from
// (object, air) exactly as the observation writer computes them, so every
// input value equals the observation's.
// K order: lane group g owns the window cells of code group g; its slot s =
// 8t + j of K-slice t holds, for s < 5 cpg, channel (s % 5 < 4 ? s % 5 : 5) of
// cell s / 5 (the 0/1 channels), and for s in [5 cpg, 6 cpg) channel 4 (charge
// / 100) of cell s - 5 cpg.  drl_qnet_pack packs layer 0's weights in the same
// order (drl_qnet_desc.input = DRL_QNET_INPUT_CODE), with the charge
// weights divided by 100 in f32: the kernel feeds the integer charge, so every
// input (0, 1 or a charge <= 100) is exact in fp16 and needs no x_lo product,
// two MFMAs per tile and slice (hi and lo weights) instead of three.  The
// products differ from W * fl(c / 100) by the rounding of fl(W / 100) and
// fl(c / 100), ~1e-7 relative: far inside the f32 act's 1e-5 bound.
// One workgroup per CU (the net fills the LDS); the kernel's ~140 VGPRs would
// leave room for 3 waves per SIMD, but __launch_bounds__ caps a workgroup at
// QN_CODE_MAXW = 8 waves (DRL_QN_CODE_WAVES is clamped to it).
#ifndef DRL_QN_CODE2_WAVES
#define DRL_QN_CODE2_WAVES 8  // drl_qnet_act_code2_kernel: 2 waves per SIMD (its ~230 VGPRs)
#endif
constexpr int QN_CODE2_WAVES = DRL_QN_CODE2_WAVES;
#ifndef DRL_QN_CODE_MAXW
#define DRL_QN_CODE_MAXW 8
#endif
constexpr int QN_CODE_MAXW = DRL_QN_CODE_MAXW;
#ifndef DRL_QN_CODE_WAVES
#define DRL_QN_CODE_WAVES 8
#endif
constexpr int QN_CODE_WAVES = DRL_QN_CODE_WAVES;

__device__ __forceinline__ float code_channel(uint32_t code, int ch) {
    const uint32_t obj = code & 7u, air = code >> 3;
    switch (ch) {
        case 0: return air ? 1.0f : 0.0f;
        case 1: return (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f;
        case 2: return obj == OBJ_DROPZONE ? 1.0f : 0.0f;
        case 3: return obj == OBJ_STATION ? 1.0f : 0.0f;
        case 4:  // the charge c itself (the observation holds c / 100; the packed weights carry the 1/100)
            return air ? (float)((int)(air & 0x7fu) - 1) : 0.0f;
        default: return obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f;
    }
}

// NT1 > 0: the net has exactly two hidden layers, the second 16 * NT1 wide
// (the benchmark's 294->128->64->5): the later layers' loops are compile-time,
// so only the live accumulators hold registers (16 waves per CU fit).
template <int NT0, bool LO0, int WN, int NT1>
__global__ void __launch_bounds__(64 * QN_CODE_MAXW) drl_qnet_act_code_kernel(QnetArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    constexpr int CPG = lay::code_cpg(WN), CPG8 = lay::code_cpg8(WN), CELLS = WN * WN;
    constexpr int NV = CPG8 / 8;                 // 16-B code vectors per lane group
    constexpr int KP = lay::code_kt(WN);         // layer 0's K-slices (host: QnetLayout::kt[0])
    static_assert(8 * KP > 6 * CPG, "no padding slot for layer 0's bias");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int c = lane & 15, g = lane >> 4;
    constexpr int nt0 = NT0;
    const int64_t ntiles = (a.E + 15) / 16;
    const int64_t gstride = (int64_t)gridDim.x * nw;
    constexpr float kLo = 1.0f / 2048.0f;
    const int ncell_g = min(CPG, CELLS - g * CPG);  // this lane group's cells (the last group may hold fewer)
    const uint4* const code = reinterpret_cast<const uint4*>(a.obs);
    auto load_codes = [&](int64_t tile, uint32_t (&dst)[4 * NV]) __attribute__((always_inline)) {
        const int64_t env = min(tile * 16 + c, a.E - 1);
        const uint4* src = code + env * (4 * NV) + g * NV;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const uint4 q = src[v];
            dst[4 * v + 0] = q.x;
            dst[4 * v + 1] = q.y;
            dst[4 * v + 2] = q.z;
            dst[4 * v + 3] = q.w;
        }
    };
#ifdef DRL_QC_STAMPS
    const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
    const int64_t grp0 = (int64_t)blockIdx.x * nw + wave;
    int64_t grp = grp0;
#ifndef DRL_DIAG_NO_WLOAD  // timing diagnostic (wrong results): no weight staging
    for (int v0 = wave * 64; v0 < a.lds_vec; v0 += 64 * nw)
        if (v0 + lane < a.lds_vec)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.packed + v0 + lane),
                                             (__attribute__((address_space(3))) void*)(wl + v0), 16, 0, 0);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool bad = false;
    const float* bias = LO0 ? reinterpret_cast<const float*>(a.packed + a.bias_vec)
                            : reinterpret_cast<const float*>(wl + a.frag_total);
    const uint4* W0 = wl + a.frag_off[0];
    const uint4* W0lo = LO0 ? wl + a.frag_lo_off[0] : a.packed + a.frag_lo_off[0];
    // the later layers' fragments and biases: global (LO0, L2-resident) by
    // buffer loads -- one VGPR of lane offset, the fragment offset in an SGPR
    // (flat loads cost a 64-bit per-lane address each) -- or the LDS image
    const auto pbuf = __builtin_amdgcn_make_buffer_rsrc((void*)a.packed, 0, a.total_bytes, 0x00020000);
    const int lane16 = lane * 16;
    auto frag_ld = [&](int frag_u4) __attribute__((always_inline)) {  // 64 lanes x 16 B at uint4 offset frag_u4
#ifdef DRL_DIAG_QC_LDS_HIDDEN  // timing diagnostic (wrong results): hidden fragments from the LDS image
        return wl[(frag_u4 & 0x3fff) + lane];
#endif
        if constexpr (LO0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, lane16, frag_u4 * 16, 0);
            uint4 r;
            __builtin_memcpy(&r, &v, 16);
            return r;
        } else {
            return wl[frag_u4 + lane];
        }
    };
    auto bias4 = [&](int off) __attribute__((always_inline)) {  // biases off + 4g .. off + 4g + 3
        f32x4 r;
#ifdef DRL_DIAG_QC_NO_BIAS  // timing diagnostic (wrong results): no bias loads
        return f32x4{0.01f * off, 0.0f, 0.0f, 0.0f};
#endif
        if constexpr (LO0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, 16 * g, a.bias_vec * 16 + off * 4, 0);
            __builtin_memcpy(&r, &v, 16);
        } else {
            const float* bp = bias + off + 4 * g;
            r = f32x4{bp[0], bp[1], bp[2], bp[3]};
        }
        return r;
    };

    uint32_t cw[4 * NV];
    load_codes(grp < ntiles ? grp : 0, cw);
    for (; grp < ntiles; grp += gstride) {
        const int64_t ngrp = grp + gstride;
        uint32_t ncw[4 * NV];  // the next tile's codes, in flight while this tile runs
        load_codes(ngrp < ntiles ? ngrp : grp, ncw);
        // the first K-slice of each layer starts its accumulators from an
        // inline zero (no zeroing moves)
        f32x4 acc[QN_MAXT], acl[QN_MAXT];
        const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
#ifdef DRL_QC_STAMPS  // diagnostic: s_memtime per phase of each wave's tiles into q (raw u32)
        const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
        for (int t = 0; t < KP; ++t) {
            const uint32_t* cs = cw;
            f16x8 bh;  // every input is 0, 1 or an integer charge <= 100: exact in fp16
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int sl = 8 * t + j;  // compile-time slot
                const int l = lay::code_slot_cell(CPG, sl), ch = lay::code_slot_ch(CPG, sl);
                float x = (sl == 6 * CPG && g == 0) ? 1.0f : 0.0f;  // the bias slot (drl_qnet_pack)
                if (sl < 6 * CPG) {
                    const uint32_t cd = (cs[l >> 1] >> (16 * (l & 1))) & 0xffffu;
#ifdef DRL_DIAG_QC_NO_DECODE  // timing diagnostics of the code act (wrong results)
                    x = (float)(cd & 1u);
#else
                    x = l < ncell_g ? code_channel(cd, ch) : 0.0f;
#endif
                }
                bh[j] = (_Float16)x;
            }
            // the slice index through an opaque SGPR: a compile-time one lets
            // LLVM hoist every fragment address (lane offset + constant, 160 of
            // them) out of the tile loop into its own VGPR
            int ts = t;
            asm volatile("" : "+s"(ts));
#pragma unroll
            for (int m = 0; m < nt0; ++m) {
                const f16x8 wh = as_f16x8(W0[(m * KP + ts) * 64 + lane]);
                const f16x8 wo = as_f16x8(W0lo[(m * KP + ts) * 64 + lane]);
#ifdef DRL_DIAG_QC_NO_L0MFMA
                acc[m] = (t == 0 ? z4 : acc[m]) + (float)bh[m] + (float)wh[0] + (float)wo[1];
                acl[m] = t == 0 ? z4 : acl[m];
#else
                acc[m] = MFMA_F16(wh, bh, t == 0 ? z4 : acc[m], 0, 0, 0);
                acl[m] = MFMA_F16(wo, bh, t == 0 ? z4 : acl[m], 0, 0, 0);
#endif
                if (m % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // <= 8 fragments in flight (registers)
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < 4 * NV; ++i) cw[i] = ncw[i];
#ifdef DRL_QC_STAMPS
        const uint64_t ts1 = __builtin_amdgcn_s_memtime();
#endif
        // ---- hidden layers and the output layer: as drl_qnet_act_f32_kernel.
        // layer(NTP, NTL, l): inputs from NTP accumulator tiles, NTL outputs
        // (compile-time bounds; the generic path passes QN_MAXT and masks)
        auto layer = [&](auto ntp_c, auto ntl_c, int l, int nt_prev, int nt_l) __attribute__((always_inline)) {
            constexpr int NTP = decltype(ntp_c)::value, NTL = decltype(ntl_c)::value;
            const int bprev = a.bias_off[l - 1];
            f16x8 ah[NTP / 2], al[NTP / 2];
#pragma unroll
            for (int s2 = 0; s2 < NTP / 2; ++s2) {
                ah[s2] = al[s2] = f16x8{};  // (not carried across layers and tiles as undefined values)
                if (2 * s2 < nt_prev) {
                    // (layer 0's bias is folded into its K padding: drl_qnet_pack)
                    const f32x4 b0 = l == 1 ? z4 : bias4(bprev + 32 * s2), b1 = l == 1 ? z4 : bias4(bprev + 32 * s2 + 16);
                    float v[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int m = 2 * s2 + (j >> 2), i = j & 3;
                        v[j] = fmaxf((acc[m][i] + acl[m][i] * kLo) + (j < 4 ? b0[i] : b1[i]), 0.0f);
                    }
                    split_f16(v, ah[s2], al[s2], bad);
                }
            }
            const int kt = nt_prev / 2, ms = kt * 64;  // (ms: the fragment stride of an output tile)
            const int fl = a.frag_off[l], flo = a.frag_lo_off[l];
#pragma unroll
            for (int t = 0; t < NTP / 2; ++t) {
                if (t < kt) {
#pragma unroll
                    for (int m = 0; m < NTL; ++m) {
                        if (m < nt_l) {
                            const f16x8 wh = as_f16x8(frag_ld(fl + m * ms + t * 64));
                            const f16x8 wo = as_f16x8(frag_ld(flo + m * ms + t * 64));
                            acc[m] = MFMA_F16(wh, ah[t], t == 0 ? z4 : acc[m], 0, 0, 0);
                            acl[m] = MFMA_F16(wh, al[t], t == 0 ? z4 : acl[m], 0, 0, 0);
                            acl[m] = MFMA_F16(wo, ah[t], acl[m], 0, 0, 0);
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // fragment reads next to their MFMAs (register pressure)
            }
        };
        int bprev;
        if constexpr (NT1 > 0) {
#ifndef DRL_DIAG_QC_NO_HIDDEN
            // every fragment of a layer requested at once, one L2 round trip
            // per layer (fragment by fragment the loads serialise on vmcnt)
            constexpr int KT1 = NT0 / 2, KT2 = NT1 / 2;
            uint4 f1h[KT1][NT1], f1l[KT1][NT1];
            {
                const int fl = a.frag_off[1], flo = a.frag_lo_off[1];
#pragma unroll
                for (int t = 0; t < KT1; ++t)
#pragma unroll
                    for (int m = 0; m < NT1; ++m) {
                        f1h[t][m] = frag_ld(fl + (m * KT1 + t) * 64);
                        f1l[t][m] = frag_ld(flo + (m * KT1 + t) * 64);
                    }
            }
            f16x8 ah[KT1], al[KT1];
#pragma unroll
            for (int s2 = 0; s2 < KT1; ++s2) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * s2 + (j >> 2), i = j & 3;
                    v[j] = fmaxf(acc[m][i] + acl[m][i] * kLo, 0.0f);  // (bias folded into layer 0)
                }
                split_f16(v, ah[s2], al[s2], bad);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < KT1; ++t)
#pragma unroll
                for (int m = 0; m < NT1; ++m) {
                    const f16x8 wh = as_f16x8(f1h[t][m]), wo = as_f16x8(f1l[t][m]);
                    acc[m] = MFMA_F16(wh, ah[t], t == 0 ? z4 : acc[m], 0, 0, 0);
                    acl[m] = MFMA_F16(wh, al[t], t == 0 ? z4 : acl[m], 0, 0, 0);
                    acl[m] = MFMA_F16(wo, ah[t], acl[m], 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
            // the output layer: fragments and layer 1's biases at once
            uint4 f2h[KT2], f2l[KT2];
            f32x4 b1[KT2][2];
            {
                const int fl = a.frag_off[2], flo = a.frag_lo_off[2], bo = a.bias_off[1];
#pragma unroll
                for (int t = 0; t < KT2; ++t) {
                    f2h[t] = frag_ld(fl + t * 64);
                    f2l[t] = frag_ld(flo + t * 64);
                    b1[t][0] = bias4(bo + 32 * t);
                    b1[t][1] = bias4(bo + 32 * t + 16);
                }
            }
            f16x8 ah2[KT2], al2[KT2];
#pragma unroll
            for (int s2 = 0; s2 < KT2; ++s2) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * s2 + (j >> 2), i = j & 3;
                    v[j] = fmaxf((acc[m][i] + acl[m][i] * kLo) + b1[s2][j >> 2][i], 0.0f);
                }
                split_f16(v, ah2[s2], al2[s2], bad);
            }
#pragma unroll
            for (int t = 0; t < KT2; ++t) {
                const f16x8 wh = as_f16x8(f2h[t]), wo = as_f16x8(f2l[t]);
                acc[0] = MFMA_F16(wh, ah2[t], t == 0 ? z4 : acc[0], 0, 0, 0);
                acl[0] = MFMA_F16(wh, al2[t], t == 0 ? z4 : acl[0], 0, 0, 0);
                acl[0] = MFMA_F16(wo, ah2[t], acl[0], 0, 0, 0);
            }
#endif
            bprev = a.bias_off[2];
        } else {
            int nt_prev = nt0;
            for (int l = 1; l <= a.n_hidden; ++l) {
                const int nt_l = (l < a.n_hidden) ? a.nt[l] : 1;
                layer(std::integral_constant<int, QN_MAXT>{}, std::integral_constant<int, QN_MAXT>{}, l, nt_prev, nt_l);
                nt_prev = nt_l;
            }
            bprev = a.bias_off[a.n_hidden];
        }
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts2 = __builtin_amdgcn_s_memtime();
#endif
        const f32x4 bq = bias4(bprev);
        float q[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float own = (acc[0][i] + acl[0][i] * kLo) + bq[i];
            const float hi = __shfl(own, c + 16);
            q[i] = own;
            q[i + 4] = hi;
        }
        const int64_t env = grp * 16 + c;
        if (g == 0 && env < a.E) {
            int best = 0;
            for (int i = 1; i < a.n_actions; ++i) best = q[i] > q[best] ? i : best;
            const uint64_t ge = (uint64_t)(a.env_offset + env);
            const uint64_t hsh = qn_splitmix64(a.seed ^ qn_splitmix64((a.step << 40) ^ (ge << 8) ^ 0xa5ull));
            const float u = (float)(hsh >> 40) * (1.0f / 16777216.0f);
            const int rnd = (int)(((hsh & 0xffffffffull) * (uint64_t)a.n_actions) >> 32);
            a.actions[env * a.action_stride] = (u < qn_eps(a)) ? rnd : best;
#ifndef DRL_QC_STAMPS
            if (a.q)
                for (int i = 0; i < a.n_actions; ++i) a.q[env * a.n_actions + i] = q[i];
#endif
        }
#ifdef DRL_QC_STAMPS
        const uint64_t ts3 = __builtin_amdgcn_s_memtime();
        if (lane == 0 && a.q) {
            uint32_t* st = reinterpret_cast<uint32_t*>(a.q) + grp * 5;
            st[0] = (uint32_t)(ts1 - ts0);
            st[1] = (uint32_t)(ts2 - ts1);
            st[2] = (uint32_t)(ts3 - ts2);
            st[3] = (uint32_t)(ts0 - t_entry);
            st[4] = (uint32_t)(ts3 - t_entry);
        }
#endif
    }
    bad |= lane == 0 && reinterpret_cast<const int32_t*>(a.packed + a.status_vec)[0] != 0;  // pack range flag
    if (__ballot(bad) && lane == 0 && a.err) atomicOr(a.err, DRL_ERR_QNET_RANGE);
    if (a.synth_n > 1) {  // as in drl_qnet_act_kernel (one 16-env tile per group)
        const uint32_t nd = (uint32_t)a.synth_n - 1u;
        const uint32_t per = 16u * nd;
        for (int64_t gg = grp0; gg < ntiles; gg += gstride) {
            for (uint32_t k = (uint32_t)lane; k < per; k += 64u) {
                const uint32_t el = k / nd;
                const int64_t env = 16 * gg + el;
                const uint64_t drone = 1u + (k - el * nd);
                if (env < a.E) {
                    const uint64_t ctr = (a.synth_step << 40) ^ ((uint64_t)(a.env_offset + env) << 8) ^ drone;
                    const uint64_t h = qn_splitmix64(a.synth_seed ^ qn_splitmix64(ctr));
                    a.actions[env * a.action_stride + (int64_t)drone] = (int32_t)(((h >> 32) * 5ull) >> 32);
                }
            }
        }
    }
}

// drl_qnet_act_code for the two-hidden-layer nets of the benchmark shape
// (NT0 = 8, NT1 = hidden[1] / 16), two 16-env tiles per wave: layer 0 is
// bound by the LDS bandwidth of its weight fragments (every tile reads the
// whole 160 KB image), so each fragment read feeds both tiles' MFMAs -- half
// the LDS bytes per env -- and each L2 fragment of the later layers serves
// both tiles.  Same arithmetic, order and results as drl_qnet_act_code_kernel.
template <int NT0, bool LO0, int WN, int NT1>
__global__ void __launch_bounds__(64 * QN_CODE2_WAVES) drl_qnet_act_code2_kernel(QnetArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    constexpr int TP = 2;
    constexpr int CPG = lay::code_cpg(WN), CPG8 = lay::code_cpg8(WN), CELLS = WN * WN;
    constexpr int NV = CPG8 / 8;                 // 16-B code vectors per lane group
    constexpr int KP = lay::code_kt(WN);         // layer 0's K-slices
    constexpr int KT1 = NT0 / 2, KT2 = NT1 / 2;  // K-slices of layer 1 and of the output layer
    static_assert(8 * KP > 6 * CPG, "no padding slot for layer 0's bias");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int c = lane & 15, g = lane >> 4;
    const int64_t ntiles = (a.E + 15) / 16;
    const int64_t ngroups = (ntiles + TP - 1) / TP;
    const int64_t gstride = (int64_t)gridDim.x * nw;
    constexpr float kLo = 1.0f / 2048.0f;
    const int ncell_g = min(CPG, CELLS - g * CPG);
    const uint4* const code = reinterpret_cast<const uint4*>(a.obs);
    auto load_codes = [&](int64_t tile, uint32_t (&dst)[4 * NV]) __attribute__((always_inline)) {
        const int64_t env = min(tile * 16 + c, a.E - 1);
        const uint4* src = code + env * (4 * NV) + g * NV;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const uint4 q = src[v];
            dst[4 * v + 0] = q.x;
            dst[4 * v + 1] = q.y;
            dst[4 * v + 2] = q.z;
            dst[4 * v + 3] = q.w;
        }
    };
    const int64_t grp0 = (int64_t)blockIdx.x * nw + wave;
    int64_t grp = grp0;
#ifdef DRL_QC_STAMPS  // diagnostic: s_memtime per phase of each wave's groups into q (raw u32, 5 per group)
    const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
    uint32_t cw[TP][4 * NV];
#pragma unroll
    for (int h = 0; h < TP; ++h) load_codes(TP * (grp < ngroups ? grp : 0) + h, cw[h]);
    for (int v0 = wave * 64; v0 < a.lds_vec; v0 += 64 * nw)
        if (v0 + lane < a.lds_vec)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.packed + v0 + lane),
                                             (__attribute__((address_space(3))) void*)(wl + v0), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool bad = false;
    const uint4* W0 = wl + a.frag_off[0];
    const uint4* W0lo = LO0 ? wl + a.frag_lo_off[0] : a.packed + a.frag_lo_off[0];
    const float* bias = LO0 ? reinterpret_cast<const float*>(a.packed + a.bias_vec)
                            : reinterpret_cast<const float*>(wl + a.frag_total);
    const auto pbuf = __builtin_amdgcn_make_buffer_rsrc((void*)a.packed, 0, a.total_bytes, 0x00020000);
    const int lane16 = lane * 16;
    auto frag_ld = [&](int frag_u4) __attribute__((always_inline)) {
        if constexpr (LO0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, lane16, frag_u4 * 16, 0);
            uint4 r;
            __builtin_memcpy(&r, &v, 16);
            return r;
        } else {
            return wl[frag_u4 + lane];
        }
    };
    auto bias4 = [&](int off) __attribute__((always_inline)) {
        f32x4 r;
        if constexpr (LO0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, 16 * g, a.bias_vec * 16 + off * 4, 0);
            __builtin_memcpy(&r, &v, 16);
        } else {
            const float* bp = bias + off + 4 * g;
            r = f32x4{bp[0], bp[1], bp[2], bp[3]};
        }
        return r;
    };
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

    for (; grp < ngroups; grp += gstride) {
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
        const int64_t ngrp = grp + gstride;
        uint32_t ncw[TP][4 * NV];  // the next group's codes, in flight while this one runs
#pragma unroll
        for (int h = 0; h < TP; ++h) load_codes(TP * (ngrp < ngroups ? ngrp : grp) + h, ncw[h]);
        // ---- layer 0: each fragment read feeds both tiles
        f32x4 acc[TP][NT0], acl[TP][NT0];
#pragma unroll
        for (int t = 0; t < KP; ++t) {
            f16x8 bh[TP];  // inputs 0, 1 or an integer charge <= 100: exact in fp16
#pragma unroll
            for (int h = 0; h < TP; ++h) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int sl = 8 * t + j;  // compile-time slot
                    const int l = lay::code_slot_cell(CPG, sl), ch = lay::code_slot_ch(CPG, sl);
                    float x = (sl == 6 * CPG && g == 0) ? 1.0f : 0.0f;  // the bias slot (drl_qnet_pack)
                    if (sl < 6 * CPG) {
                        const uint32_t cd = (cw[h][l >> 1] >> (16 * (l & 1))) & 0xffffu;
                        x = l < ncell_g ? code_channel(cd, ch) : 0.0f;
                    }
                    bh[h][j] = (_Float16)x;
                }
            }
            int ts = t;  // opaque slice index (see drl_qnet_act_code_kernel)
            asm volatile("" : "+s"(ts));
#pragma unroll
            for (int m = 0; m < NT0; ++m) {
                const f16x8 wh = as_f16x8(W0[(m * KP + ts) * 64 + lane]);
                const f16x8 wo = as_f16x8(W0lo[(m * KP + ts) * 64 + lane]);
#pragma unroll
                for (int h = 0; h < TP; ++h) {
                    acc[h][m] = MFMA_F16(wh, bh[h], t == 0 ? z4 : acc[h][m], 0, 0, 0);
                    acl[h][m] = MFMA_F16(wo, bh[h], t == 0 ? z4 : acl[h][m], 0, 0, 0);
                }
                if (m % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // <= 8 fragments in flight
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int h = 0; h < TP; ++h)
#pragma unroll
            for (int i = 0; i < 4 * NV; ++i) cw[h][i] = ncw[h][i];
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts1 = __builtin_amdgcn_s_memtime();
#endif
        // ---- layer 1 (bias folded into layer 0): inputs as fp16 hi/lo
        f16x8 ah[TP][KT1], al[TP][KT1];
#pragma unroll
        for (int h = 0; h < TP; ++h)
#pragma unroll
            for (int s2 = 0; s2 < KT1; ++s2) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * s2 + (j >> 2), i = j & 3;
                    v[j] = fmaxf(acc[h][m][i] + acl[h][m][i] * kLo, 0.0f);
                }
                split_f16(v, ah[h][s2], al[h][s2], bad);
            }
        f32x4 bcc[TP][NT1], bcl[TP][NT1];
        {
            const int fl = a.frag_off[1], flo = a.frag_lo_off[1];
#pragma unroll
            for (int t0 = 0; t0 < KT1; ++t0) {  // a K-slice's fragments at once (two: spills)
                uint4 fh[1][NT1], fo[1][NT1];
#pragma unroll
                for (int u = 0; u < 1; ++u)
#pragma unroll
                    for (int m = 0; m < NT1; ++m) {
                        fh[u][m] = frag_ld(fl + (m * KT1 + t0 + u) * 64);
                        fo[u][m] = frag_ld(flo + (m * KT1 + t0 + u) * 64);
                    }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 1; ++u)
#pragma unroll
                    for (int m = 0; m < NT1; ++m) {
                        const int t = t0 + u;
                        const f16x8 wh = as_f16x8(fh[u][m]), wo = as_f16x8(fo[u][m]);
#pragma unroll
                        for (int h = 0; h < TP; ++h) {
                            bcc[h][m] = MFMA_F16(wh, ah[h][t], t == 0 ? z4 : bcc[h][m], 0, 0, 0);
                            bcl[h][m] = MFMA_F16(wh, al[h][t], t == 0 ? z4 : bcl[h][m], 0, 0, 0);
                            bcl[h][m] = MFMA_F16(wo, ah[h][t], bcl[h][m], 0, 0, 0);
                        }
                    }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts2 = __builtin_amdgcn_s_memtime();
#endif
        // ---- the output layer: fragments and layer 1's biases at once
        uint4 f2h[KT2], f2l[KT2];
        f32x4 b1[KT2][2];
        {
            const int fl = a.frag_off[2], flo = a.frag_lo_off[2], bo = a.bias_off[1];
#pragma unroll
            for (int t = 0; t < KT2; ++t) {
                f2h[t] = frag_ld(fl + t * 64);
                f2l[t] = frag_ld(flo + t * 64);
                b1[t][0] = bias4(bo + 32 * t);
                b1[t][1] = bias4(bo + 32 * t + 16);
            }
        }
        const f32x4 bq = bias4(a.bias_off[2]);
#pragma unroll
        for (int h = 0; h < TP; ++h) {
            f16x8 ah2[KT2], al2[KT2];
#pragma unroll
            for (int s2 = 0; s2 < KT2; ++s2) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * s2 + (j >> 2), i = j & 3;
                    v[j] = fmaxf((bcc[h][m][i] + bcl[h][m][i] * kLo) + b1[s2][j >> 2][i], 0.0f);
                }
                split_f16(v, ah2[s2], al2[s2], bad);
            }
            f32x4 qc, ql;
#pragma unroll
            for (int t = 0; t < KT2; ++t) {
                const f16x8 wh = as_f16x8(f2h[t]), wo = as_f16x8(f2l[t]);
                qc = MFMA_F16(wh, ah2[t], t == 0 ? z4 : qc, 0, 0, 0);
                ql = MFMA_F16(wh, al2[t], t == 0 ? z4 : ql, 0, 0, 0);
                ql = MFMA_F16(wo, ah2[t], ql, 0, 0, 0);
            }
            float q[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float own = (qc[i] + ql[i] * kLo) + bq[i];
                const float hi = __shfl(own, c + 16);
                q[i] = own;
                q[i + 4] = hi;
            }
            const int64_t env = (TP * grp + h) * 16 + c;
            if (g == 0 && env < a.E) {
                int best = 0;
                for (int i = 1; i < a.n_actions; ++i) best = q[i] > q[best] ? i : best;
                const uint64_t ge = (uint64_t)(a.env_offset + env);
                const uint64_t hsh = qn_splitmix64(a.seed ^ qn_splitmix64((a.step << 40) ^ (ge << 8) ^ 0xa5ull));
                const float u = (float)(hsh >> 40) * (1.0f / 16777216.0f);
                const int rnd = (int)(((hsh & 0xffffffffull) * (uint64_t)a.n_actions) >> 32);
                a.actions[env * a.action_stride] = (u < qn_eps(a)) ? rnd : best;
#ifndef DRL_QC_STAMPS
                if (a.q)
                    for (int i = 0; i < a.n_actions; ++i) a.q[env * a.n_actions + i] = q[i];
#endif
            }
        }
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts3 = __builtin_amdgcn_s_memtime();
        if (lane == 0 && a.q) {
            uint32_t* st = reinterpret_cast<uint32_t*>(a.q) + grp * 5;
            st[0] = (uint32_t)(ts1 - ts0);
            st[1] = (uint32_t)(ts2 - ts1);
            st[2] = (uint32_t)(ts3 - ts2);
            st[3] = (uint32_t)(ts0 - t_entry);
            st[4] = (uint32_t)(ts3 - t_entry);
        }
#endif
    }
    bad |= lane == 0 && reinterpret_cast<const int32_t*>(a.packed + a.status_vec)[0] != 0;  // pack range flag
    if (__ballot(bad) && lane == 0 && a.err) atomicOr(a.err, DRL_ERR_QNET_RANGE);
    if (a.synth_n > 1) {  // as in drl_qnet_act_kernel (TP 16-env tiles per group)
        const uint32_t nd = (uint32_t)a.synth_n - 1u;
        const uint32_t per = (uint32_t)(TP * 16) * nd;
        for (int64_t gg = grp0; gg < ngroups; gg += gstride) {
            for (uint32_t k = (uint32_t)lane; k < per; k += 64u) {
                const uint32_t el = k / nd;
                const int64_t env = TP * 16 * gg + el;
                const uint64_t drone = 1u + (k - el * nd);
                if (env < a.E) {
                    const uint64_t ctr = (a.synth_step << 40) ^ ((uint64_t)(a.env_offset + env) << 8) ^ drone;
                    const uint64_t hh = qn_splitmix64(a.synth_seed ^ qn_splitmix64(ctr));
                    a.actions[env * a.action_stride + (int64_t)drone] = (int32_t)(((hh >> 32) * 5ull) >> 32);
                }
            }
        }
    }
}

// ------------------------------------- inline LDS reads of the code act ---
// Helpers of drl_qnet_act_code4_kernel (round 3's v3 kernel, whose measured
// lessons v4 builds on, is described in DESIGN.md; removed in round 5): a
// compile-time loop, fragment reads as inline ds_read_b128 with explicit
// lgkmcnt waits (the compiler would otherwise put a vmcnt(0) for the LDS-DMA
// in front of the first LDS read and drain the whole staging before any MFMA).
typedef uint32_t q3u4 __attribute__((ext_vector_type(4)));

template <int I, int N, class F>
__device__ __forceinline__ void qc3_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        qc3_for<I + 1, N>(f);
    }
}

template <int OFF>
__device__ __forceinline__ void qc3_read(q3u4& r, const uint32_t (&base)[3]) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base[OFF >> 16]), "i"(OFF & 0xffff));
}

template <int N>
__device__ __forceinline__ void qc3_wait(q3u4& r) {  // this fragment's read has landed (later reads may not)
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r) : "i"(N));
}

__device__ __forceinline__ f16x8 q3_f16(const q3u4 v) {
    f16x8 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}

// ------------------------------------------------ act from the code, v4 ---
// drl_qnet_act_code4_kernel: the benchmark nets (layer 0's hi + lo fragments
// the LDS image, 8 unit tiles, two hidden layers, the second 16 * NT1 wide) at
// ONE wave per SIMD: four waves per workgroup, one workgroup per CU, 512
// registers per wave, four 16-env tiles (64 envs) per wave pass.
// What the v3 kernel (two waves per SIMD, two tiles) and the first v4 showed
// (profiles/r04_act/): staging the 160 KB image on every CU costs about
// nothing (tools/stage_probe: an LDS-DMA kernel staging 160 KB per CU times
// like an empty launch); the phases were VALU-bound, not MFMA- or LDS-bound:
// per 64-env pass, layer 0 issued 1,346 VALU beside its 640 MFMAs (the
// per-slot channel decode, ~6 instructions per K slot), layer 1 892 beside 192
// (the f32 -> fp16 hi/lo split), the output layer and the epilogue 1,127 (the
// split again, the exploration hash and per-tile epilogues on 16 of 64 lanes).
// With one wave per SIMD an MFMA leaves room for about two VALU instructions,
// so this kernel
//  * decodes the code two slots per instruction: the K order (lay::code_slot_*)
//    makes a dword of the B operand one channel of one code dword (two cells),
//    computed with packed 16-bit operations: the object channels by one
//    v_perm_b32 lookup each (fp16 1.0's high byte 0x3C in a byte table indexed
//    by the object), the drone flag by a min and a multiply, the charge by a
//    saturating subtract and the fp16 magic 1024 + n; one dword per step (four
//    MFMAs), the lo inputs (x * 2^-11, exact) beside it;
//  * splits with v_cvt_pk_f16_f32 and checks the range through a running
//    maximum (one compare per pass instead of one per value), the next K
//    slice's split beside the current slice's MFMAs;
//  * computes the exploration draw (two splitmix64) at the start of the pass
//    and runs the argmax once per pass on all 64 lanes: lane (c, g) takes env c
//    of tile g, its Q rows gathered with shuffles.
#ifndef DRL_QC4_PD
#define DRL_QC4_PD 6
#endif
constexpr int QC4_PD = DRL_QC4_PD;  // layer-0 fragment reads in flight per wave (ring of QC4_PD + 2)
constexpr int QC4_WAVES = 4;
#ifndef DRL_QC4_PIN
#define DRL_QC4_PIN 0  // A/B knob: empty-asm pins keeping each step's decode between its MFMAs
#endif
#ifndef DRL_QC4_EARLYVEC
#define DRL_QC4_EARLYVEC 0  // A/B knob: slice 0 waits only for the first code vector of each tile
#endif
#ifndef DRL_QC4_DMALOOP
#define DRL_QC4_DMALOOP 0  // A/B knob: stage slices >= 2 inside layer 0 (measured slower: 17.6 vs 16.5 us at C3)
#endif
#ifndef DRL_QC4_XCD
#define DRL_QC4_XCD 0  // A/B knob: XCD-contiguous env groups (with the step's DRL_XCD_REMAP: codes read from the L2 they were written to)
#endif
#ifndef DRL_QC4_EARLYSPLIT
#define DRL_QC4_EARLYSPLIT 1  // layer 1's first split inside layer 0's last slice (16.33-16.53 vs 16.44-16.75 us, g19)
#endif
#ifndef DRL_QC4_EARLYNEXT
#define DRL_QC4_EARLYNEXT 0  // A/B knob: the second pass's codes loaded in the prologue (C5 act in the loop 41.4 vs 42.0 us, C3 loop 45.8 vs 45.1-45.4: not kept)
#endif
#ifndef DRL_QC4_IGLP1
#define DRL_QC4_IGLP1 0  // A/B knob: sched_group_barrier MFMA / 3 VALU interleave of layer 1
#endif
#ifndef DRL_QC4_IGLP
#define DRL_QC4_IGLP 0  // A/B knob: sched_group_barrier MFMA / 2 VALU interleave per step
#endif

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <class T, class F>
__device__ __forceinline__ T qc4_as(const F v) {
    static_assert(sizeof(T) == sizeof(F), "bit cast");
    T r;
    __builtin_memcpy(&r, &v, sizeof(T));
    return r;
}

// object channels: v_perm_b32 byte tables (bytes 0-3 from the second operand, 4-7 from the first) with
// 0x3C at the object's code; selector: byte 1 (3) = the object of the dword's low (high) cell, bytes 0 and 2
// = 0x0C (a zero byte)
__device__ __forceinline__ uint32_t qc4_obj_sel(uint32_t w) { return ((w & 0x00070007u) << 8) | 0x000C000Cu; }
template <int OBJ>
__device__ __forceinline__ uint32_t qc4_obj(uint32_t sel) {
    constexpr uint32_t hi = OBJ >= 4 ? 0x3Cu << (8 * (OBJ - 4)) : 0u, lo = OBJ < 4 ? 0x3Cu << (8 * OBJ) : 0u;
    return __builtin_amdgcn_perm(hi, lo, sel);
}
// channel CH (wrappers.py:10-31, code_channel) of both cells of code dword w, as two fp16 (the charge as the
// integer c: the packed weights carry the 1/100)
template <int CH>
__device__ __forceinline__ uint32_t qc4_channel(uint32_t w) {
    if constexpr (CH == 0) {  // a drone: air != 0, i.e. (charge + 1) != 0 in bits 3-9
        const u16x2 m = __builtin_elementwise_min(qc4_as<u16x2>(w & 0x03F803F8u), (u16x2){8, 8});
        return qc4_as<uint32_t>(m * (u16x2){0x780, 0x780});  // 8 * 0x780 = 0x3C00
    } else if constexpr (CH == 1) {  // a packet on the ground or carried
        const u16x2 cr = qc4_as<u16x2>(w & 0x04000400u) * (u16x2){15, 15};  // 0x400 * 15 = 0x3C00
        return qc4_obj<OBJ_PACKET>(qc4_obj_sel(w)) | qc4_as<uint32_t>(cr);
    } else if constexpr (CH == 2) {
        return qc4_obj<OBJ_DROPZONE>(qc4_obj_sel(w));
    } else if constexpr (CH == 3) {
        return qc4_obj<OBJ_STATION>(qc4_obj_sel(w));
    } else if constexpr (CH == 4) {  // the charge c = (air & 0x7f) - 1 (0 without a drone), as fp16 (1024 + c) - 1024
        const u16x2 c1 = qc4_as<u16x2>((w >> 3) & 0x007F007Fu);
        const u16x2 c = __builtin_elementwise_sub_sat(c1, (u16x2){1, 1});
        const f16x2 f = qc4_as<f16x2>(qc4_as<uint32_t>(c) | 0x64006400u);
        return qc4_as<uint32_t>(f - (f16x2){(_Float16)1024.0f, (_Float16)1024.0f});
    } else {
        return qc4_obj<OBJ_SKYSCRAPER>(qc4_obj_sel(w));
    }
}
template <int CH>
__device__ __forceinline__ uint32_t qc4_channel_lo16(uint32_t w) {  // channel CH of the dword's low cell only
    return qc4_channel<CH>(w & 0xffffu) & 0xffffu;
}

// B dword D (slots 2D, 2D + 1) of a lane group's K order from the code word qc4_word<CPG, D> of its
// CPG cells (two per word)
template <int CPG, int D>
constexpr int qc4_word() { return D < 6 * (CPG / 2) ? D / 6 : CPG / 2; }
template <int CPG, int D>
__device__ __forceinline__ uint32_t qc4_bdword(const uint32_t w, bool bias_group) {
    constexpr int NP = CPG / 2;  // cell pairs
    if constexpr (D < 6 * NP) {
        return qc4_channel<D % 6>(w);
    } else if constexpr (D < 3 * CPG) {  // the odd count's last cell (the low half of its code word): two channels
        constexpr int ch = 2 * (D - 6 * NP);
        return qc4_channel_lo16<ch>(w) | (qc4_channel_lo16<ch + 1>(w) << 16);
    } else if constexpr (D == 3 * CPG) {  // slot 6 * CPG: the bias (input 1.0 in lane group 0)
        return bias_group ? 0x3C00u : 0u;
    } else {
        return 0u;
    }
}

// ReLU of an f32 as an integer max on its bits (negative floats are negative ints: no NaN canonicalisation, one
// instruction); the split of 8 ReLU'd activations into fp16 hi = fp16(r) (v_cvt_pk_f16_f32) and lo =
// fp16((r - hi) * 2^11) (v_fma_mix{lo,hi}_f16 on hi and r * 2^11: one rounding of the exact difference), and the
// running maximum of the activations' bits (non-negative floats order as unsigned ints) for the range flag
__device__ __forceinline__ float qc4_relu(float v) {
    return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int32_t, v), 0));
}
__device__ __forceinline__ void qc4_split(const float (&r)[8], f16x8& hi, f16x8& lo, uint32_t& mx) {
    const float m2k = -2048.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float a = r[2 * k], b = r[2 * k + 1];
        const f16x2 h = {(_Float16)a, (_Float16)b};
        const uint32_t hw = qc4_as<uint32_t>(h);
        uint32_t lw;
        asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=&v"(lw) : "v"(hw), "v"(m2k), "v"(a * 2048.0f));
        asm("v_fma_mixhi_f16 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "+v"(lw) : "v"(hw), "v"(m2k), "v"(b * 2048.0f));
        const f16x2 l = qc4_as<f16x2>(lw);
        hi[2 * k] = h[0];
        hi[2 * k + 1] = h[1];
        lo[2 * k] = l[0];
        lo[2 * k + 1] = l[1];
        mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(__builtin_bit_cast(uint32_t, a),
                                                                     __builtin_bit_cast(uint32_t, b)));
    }
}

template <int NT0, int WN, int NT1>
__global__ void __launch_bounds__(64 * QC4_WAVES) __attribute__((amdgpu_waves_per_eu(1, 1)))
drl_qnet_act_code4_kernel(QnetArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    constexpr int TP = 4, NW = QC4_WAVES;
    constexpr int CPG = lay::code_cpg(WN), CPG8 = lay::code_cpg8(WN);
    constexpr int NV = CPG8 / 8;                 // 16-B code vectors per lane group
    constexpr int KP = lay::code_kt(WN);         // layer 0's K-slices
    constexpr int KT1 = NT0 / 2, KT2 = NT1 / 2;  // K-slices of layer 1 and of the output layer
    constexpr int SPS = 2 * NT0;                 // steps (fragment reads) per slice: hi m = 0.., then lo m = 0..
    constexpr int STEPS = KP * SPS;
    constexpr int PD = QC4_PD, RS = PD + 2;
    constexpr int FLO = NT0 * KP * 64;           // uint4 offset of the lo fragments (lo0_lds layout)
    static_assert(8 * KP > 6 * CPG, "no padding slot for layer 0's bias");
    static_assert(2 * FLO * 16 <= 160 * 1024, "layer 0 must fit the LDS");
    static_assert(NT0 == 2 * NW, "wave w stages unit tiles 2w and 2w + 1");
    static_assert(SPS == 4 * TP, "one B dword of one tile per step: 4 dwords x TP tiles per slice");
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 15, g = lane >> 4;
    const int64_t ntiles = (a.E + 15) / 16;
    const int64_t ngroups = (ntiles + TP - 1) / TP;
#if DRL_QC4_XCD
    // (A/B) XCD-contiguous groups: the workgroups of XCD x (blockIdx % 8 == x) take a contiguous eighth of the
    // groups, each wave its passes at stride NW -- the envs whose codes a step built with DRL_XCD_REMAP wrote
    // on the same XCD (its L2)
    const int64_t passes = (ngroups + (int64_t)gridDim.x * NW - 1) / ((int64_t)gridDim.x * NW);
    const uint32_t bq = gridDim.x / 8, br = gridDim.x % 8, bxx = blockIdx.x % 8;
    const int64_t bx = (int64_t)((bxx < br ? bxx * (bq + 1) : br * (bq + 1) + (bxx - br) * bq) + blockIdx.x / 8);
    const int64_t gstride = NW;
    const int64_t gend = min(ngroups, (bx + 1) * NW * passes);
#else
    const int64_t gstride = (int64_t)gridDim.x * NW;
    const int64_t gend = ngroups;
#endif
    constexpr float kLo = 1.0f / 2048.0f;
    const f16x2 kLo2 = {(_Float16)kLo, (_Float16)kLo};
    // the codes through a buffer resource: 32-bit lane offsets (the launch keeps E * code bytes < 2^31), so no
    // 64-bit lane address stays live across layer 0 for the next pass's loads
    const auto crsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.obs, 0, (int)(a.E * (64 * NV)), 0x00020000);
    auto load_vec = [&](int64_t tile, int v, uint32_t (&dst)[4 * NV]) __attribute__((always_inline)) {
        uint32_t ln;  // the lane index, recomputed here (opaque): nothing lane-dependent is kept for these loads
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const uint32_t env = (uint32_t)min(tile * 16 + (int64_t)(ln & 15u), a.E - 1);
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(
            crsrc, (int)(env * (64u * NV) + ((ln >> 4) * NV + (uint32_t)v) * 16u), 0, 0);
        uint4 q;
        __builtin_memcpy(&q, &r, 16);
        dst[4 * v + 0] = q.x;
        dst[4 * v + 1] = q.y;
        dst[4 * v + 2] = q.z;
        dst[4 * v + 3] = q.w;
    };
    auto load_codes = [&](int64_t tile, uint32_t (&dst)[4 * NV]) __attribute__((always_inline)) {
#pragma unroll
        for (int v = 0; v < NV; ++v) load_vec(tile, v, dst);
    };
#if DRL_QC4_XCD
    const int64_t grp0 = bx * NW * passes + wave;
#else
    const int64_t grp0 = (int64_t)blockIdx.x * NW + wave;
#endif
#ifdef DRL_QC_STAMPS
    const uint64_t t_entry = __builtin_amdgcn_s_memtime();
#endif
    const auto pbuf = __builtin_amdgcn_make_buffer_rsrc((void*)a.packed, 0, a.total_bytes, 0x00020000);
    const int lane16 = lane * 16;
    auto frag_ld = [&](int frag_u4) __attribute__((always_inline)) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, lane16, frag_u4 * 16, 0);
        uint4 r;
        __builtin_memcpy(&r, &v, 16);
        return r;
    };
    auto bias4 = [&](int off) __attribute__((always_inline)) {
        f32x4 r;
        uint32_t ln;  // (the lane index recomputed, opaque: its offset is not kept in a register across layer 0)
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(pbuf, (int)((ln >> 4) * 16u), a.bias_vec * 16 + off * 4, 0);
        __builtin_memcpy(&r, &v, 16);
        return r;
    };
    // the output layer's fragments and biases (loaded during layer 1)
    auto ld2 = [&](uint4 (&f2h)[KT2], uint4 (&f2l)[KT2], f32x4 (&b1)[KT2][2], f32x4& bq) __attribute__((always_inline)) {
        const int fl = a.frag_off[2], flo = a.frag_lo_off[2], bo = a.bias_off[1];
#pragma unroll
        for (int u = 0; u < KT2; ++u) {
            f2h[u] = frag_ld(fl + u * 64);
            f2l[u] = frag_ld(flo + u * 64);
            b1[u][0] = bias4(bo + 32 * u);
            b1[u][1] = bias4(bo + 32 * u + 16);
        }
        bq = bias4(a.bias_off[2]);
    };
    // staging in slice order: wave w copies unit tiles 2w and 2w + 1, hi and lo (4 fragments per slice).
    // Slices < KE go before the codes; one forced vmcnt(0) covers them and the codes (the compiler would wait
    // for an LDS-DMA with vmcnt(0) anyway), then the other slices.
    auto dma = [&](int t) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int v0 = h * FLO + ((2 * wave + u) * KP + t) * 64;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.packed + v0 + lane),
                                                 (__attribute__((address_space(3))) void*)(wl + v0), 16, 0, 0);
            }
    };
    // issue order: every tile's first code vector (the inputs of slices 0..5 at a 7x7 window), slices 0 and 1,
    // the other code vectors, the other slices; slice t is readable once this wave's loads up to its DMAs have
    // landed (in-order vmcnt) and every wave's (the barrier)
    constexpr int KE = KP < 2 ? KP : 2;
    uint32_t cw[TP][4 * NV];
    const int64_t gl0 = grp0 < gend ? grp0 : 0;
#if DRL_QC4_EARLYVEC
#pragma unroll
    for (int h = 0; h < TP; ++h) load_vec(TP * gl0 + h, 0, cw[h]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < KE; ++t) dma(t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int v = 1; v < NV; ++v)
#pragma unroll
        for (int h = 0; h < TP; ++h) load_vec(TP * gl0 + h, v, cw[h]);
    constexpr int NE0 = 4 * (KP - KE) + TP * (NV - 1);  // vector ops younger than the slice-0 inputs
#else
#pragma unroll
    for (int t = 0; t < KE; ++t) dma(t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < TP; ++h) load_codes(TP * gl0 + h, cw[h]);
#pragma unroll
    for (int h = 0; h < TP; ++h)
#pragma unroll
        for (int i = 0; i < 4 * NV; ++i) asm volatile("s_waitcnt vmcnt(0)" : "+v"(cw[h][i]));
    constexpr int NE0 = 4 * (KP - KE);
#endif
    __builtin_amdgcn_sched_barrier(0);
#if DRL_QC4_DMALOOP
    // slices >= KE are staged inside the first pass's layer 0: slice s's four fragments at steps 1, 5, 9, 13 of
    // slice s - 2 (one LDS-DMA instruction holds the issuing wave ~60-180 cycles: all 32 in the prologue kept
    // every wave ~5k cycles from its first MFMA).  slice_ready(T) runs at step 16 T - PD, when slice T + 1's
    // fragments issued at steps <= 16 - PD of slice T - 1 are younger than slice T's.
    static_assert(!DRL_QC4_EARLYVEC && KE == 2, "DMALOOP stages slices >= 2 in the loop");
    constexpr int NDY = (1 <= 16 - PD) + (5 <= 16 - PD) + (9 <= 16 - PD) + (13 <= 16 - PD);
    if (grp0 >= gend) {  // a wave without a pass still stages its fragments
#pragma unroll
        for (int t = KE; t < KP; ++t) dma(t);
    }
#else
#pragma unroll
    for (int t = KE; t < KP; ++t) dma(t);
#endif
    __builtin_amdgcn_sched_barrier(0);
    uint32_t ncw[TP][4 * NV];  // the next pass's codes
#if DRL_QC4_EARLYNEXT
    // the second pass's codes, youngest of the prologue's loads (the slice waits below count them), in flight from
    // the start: in the train loop they come from HBM, and a prefetch during the first pass's layer 1 left their
    // latency exposed at the second pass's start (C5 act 42 us in the loop against 28 back to back).
    // Unconditional (past the last pass the first pass's again, from L2), so every wait count is static.
#pragma unroll
    for (int h = 0; h < TP; ++h) load_codes(TP * (grp0 + gstride < gend ? grp0 + gstride : gl0) + h, ncw[h]);
    constexpr int NNX = TP * NV;
#else
    constexpr int NNX = 0;
#endif
    __builtin_amdgcn_sched_barrier(0);
    auto slice_ready = [&](auto t_c) __attribute__((always_inline)) {
        constexpr int T = decltype(t_c)::value;
#if DRL_QC4_DMALOOP
        constexpr int N = T == 0 ? 0 : (T + 1 < KP ? NDY : 0);
#else
        constexpr int N = (T < KE ? NE0 : 4 * (KP - 1 - T)) + NNX;
#endif
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
    };
    uint32_t mx = 0;  // bits of the largest activation split into fp16 (DRL_ERR_QNET_RANGE at >= 65520)
    const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t base[3] = {(uint32_t)lane16, (uint32_t)lane16 + 65536u, (uint32_t)lane16 + 131072u};
    const bool bias_group = g == 0;

    bool first = true;
    if (grp0 >= gend) {  // no group: still take part in the staging barriers
        qc3_for<0, KP>([&](auto t_c) { slice_ready(t_c); });
    }
    for (int64_t grp = grp0; grp < gend; grp += gstride) {
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
        const int64_t ngrp = grp + gstride;
        const int64_t env = (TP * grp + g) * 16 + c;  // the env whose action this lane writes (tile g, column c)
#ifdef DRL_QC_STAMPS
        uint32_t slice_ts[KP];
#endif
        f32x4 acc[TP][NT0];
        uint32_t bh[2][TP][4], bl[2][TP][4];  // B operands: [slice parity][tile][dword]
        q3u4 ring[RS];
        if (first) slice_ready(std::integral_constant<int, 0>{});  // (the codes of slice 0 too)
        qc3_for<0, 4>([&](auto d_c) {
            constexpr int D = decltype(d_c)::value;
#pragma unroll
            for (int h = 0; h < TP; ++h) {
                bh[0][h][D] = qc4_bdword<CPG, D>(cw[h][qc4_word<CPG, D>()], bias_group);
                bl[0][h][D] = qc4_as<uint32_t>(qc4_as<f16x2>(bh[0][h][D]) * kLo2);
            }
        });
        // the exploration draw (independent of Q): rnd when u < epsilon, else -1
        int explore;
        {
            const uint64_t ge = (uint64_t)(a.env_offset + env);
            const uint64_t hsh = qn_splitmix64(a.seed ^ qn_splitmix64((a.step << 40) ^ (ge << 8) ^ 0xa5ull));
            const float u = (float)(hsh >> 40) * (1.0f / 16777216.0f);
            const int rnd = (int)(((hsh & 0xffffffffull) * (uint64_t)a.n_actions) >> 32);
            explore = (u < qn_eps(a)) ? rnd : -1;
        }
        uint4 f1[2][2][NT1];  // layer 1's fragments: [buffer][hi / lo][unit tile]
        uint4 f2h[KT2], f2l[KT2];  // the output layer's, and the biases
        f32x4 b1[KT2][2], bq;
        auto ld1 = [&](int t, int b) __attribute__((always_inline)) {
            const int fl = a.frag_off[1], flo = a.frag_lo_off[1];
#pragma unroll
            for (int m = 0; m < NT1; ++m) {
                f1[b][0][m] = frag_ld(fl + (m * KT1 + t) * 64);
                f1[b][1][m] = frag_ld(flo + (m * KT1 + t) * 64);
            }
        };
        f16x8 ah[2][TP], al[2][TP];  // layer 1's inputs: [K-slice parity][tile]
        auto split1_tile = [&](int t, int b, int h) __attribute__((always_inline)) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = qc4_relu(acc[h][2 * t + (j >> 2)][j & 3]);
            qc4_split(v, ah[b][h], al[b][h], mx);
        };
        auto split1 = [&](int t, int b) __attribute__((always_inline)) {
#pragma unroll
            for (int h = 0; h < TP; ++h) split1_tile(t, b, h);
        };
        // ---- layer 0: STEPS fragment reads, PD ahead of their MFMAs
        auto issue = [&](auto s_c) __attribute__((always_inline)) {
            constexpr int S = decltype(s_c)::value;
            if constexpr (S < STEPS) {
                constexpr int t = S / SPS, hl = (S / NT0) & 1, m = S % NT0;
                if constexpr (S % SPS == 0 && t > 0) {
                    if (first) slice_ready(std::integral_constant<int, t>{});
                }
                qc3_read<(hl * FLO + (m * KP + t) * 64) * 16>(ring[S % RS], base);
            }
        };
        qc3_for<0, PD>([&](auto s_c) { issue(s_c); });
        qc3_for<0, STEPS>([&](auto s_c) {
            constexpr int S = decltype(s_c)::value;
            constexpr int t = S / SPS, st = S % SPS, hl = (S / NT0) & 1, m = S % NT0;
            constexpr int after = (S + PD - 1 < STEPS ? S + PD - 1 : STEPS - 1) - S;
            qc3_wait<after>(ring[S % RS]);
            const f16x8 w = q3_f16(ring[S % RS]);
#pragma unroll
            for (int h = 0; h < TP; ++h) {
                f16x8 x;
                __builtin_memcpy(&x, hl ? bl[t & 1][h] : bh[t & 1][h], 16);
                acc[h][m] = MFMA_F16(w, x, (t == 0 && hl == 0) ? z4 : acc[h][m], 0, 0, 0);
            }
#if DRL_QC4_DMALOOP
            if constexpr (t + 2 < KP && (st == 1 || st == 5 || st == 9 || st == 13)) {  // slice t + 2's fragment
                if (first) {  // (through the buffer resource: a uniform offset, no 64-bit lane address)
                    constexpr int k = st / 4, h = k >> 1, u = k & 1;
                    const int v0 = h * FLO + ((2 * wave + u) * KP + t + 2) * 64;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(pbuf, (__attribute__((address_space(3))) void*)(wl + v0), 16,
                                                             lane16, v0 * 16, 0, 0);
                }
            }
#endif
            issue(std::integral_constant<int, S + PD>{});
            if constexpr (t + 1 < KP) {  // dword st % 4 of tile st / 4 of the next slice's inputs, pinned to this
                // step (empty asm on its input and outputs) so that it issues between this step's MFMAs
                constexpr int h = st / 4, dd = st % 4, D = 4 * (t + 1) + dd;
                uint32_t w = cw[h][qc4_word<CPG, D>()];
#if DRL_QC4_PIN
                asm volatile("" : "+v"(w));
#endif
#ifdef DRL_DIAG_QC4_NODECODE  // timing diagnostic (wrong results): no channel decode in the loop
                uint32_t xh = w;
#else
                uint32_t xh = qc4_bdword<CPG, D>(w, bias_group);
#endif
                uint32_t xl = qc4_as<uint32_t>(qc4_as<f16x2>(xh) * kLo2);
#if DRL_QC4_PIN
                asm volatile("" : "+v"(xh), "+v"(xl));
#endif
                bh[(t + 1) & 1][h][dd] = xh;
                bl[(t + 1) & 1][h][dd] = xl;
            }
            // the last slice: layer 1's first fragments and the output layer's weights (the next pass's codes
            // follow in layer 1, after ld1(1): waiting for f1[0] then waits for neither)
            if constexpr (t + 1 == KP && st == 3) ld1(0, 0);
            if constexpr (t + 1 == KP && st == 6) ld2(f2h, f2l, b1, bq);
#if DRL_QC4_EARLYSPLIT
            // layer 1's first K-slice reads unit tiles 0 and 1, final after this slice's steps 8 and 9: tile
            // st - 11's split beside the last steps' MFMAs
            if constexpr (t + 1 == KP && st >= 11 && st - 11 < TP) split1_tile(0, 0, st - 11);
#endif
#if DRL_QC4_IGLP
#pragma unroll
            for (int i = 0; i < TP; ++i) {  // one MFMA, then two VALU, per MFMA of the step
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
#endif
#ifdef DRL_QC_STAMPS
            if constexpr (st == SPS - 1) slice_ts[t] = (uint32_t)(__builtin_amdgcn_s_memtime() - ts0);
#endif
            __builtin_amdgcn_sched_barrier(0);
        });
        first = false;
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts1 = __builtin_amdgcn_s_memtime();
#endif
        // ---- layer 1 (bias folded into layer 0); K-slice t's inputs split from layer 0's unit tiles 2t, 2t + 1,
        // the next slice's split beside this slice's MFMAs
        f32x4 bcc[TP][NT1], bcl[TP][NT1];
#if !DRL_QC4_EARLYSPLIT
        split1(0, 0);
#endif
#pragma unroll
        for (int t = 0; t < KT1; ++t) {
            if (t + 1 < KT1) ld1(t + 1, (t + 1) & 1);
            if (t + 1 == KT1 && ngrp < gend && !(DRL_QC4_EARLYNEXT && grp == grp0)) {  // the next pass's codes (the
                // first pass's successor was loaded in the prologue), into their own registers and younger than
                // every layer-1 fragment (the compiler's wait counts for those then ignore them); copied at the end
#pragma unroll
                for (int h = 0; h < TP; ++h) load_codes(TP * ngrp + h, ncw[h]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < NT1; ++m) {
                const f16x8 wh = as_f16x8(f1[t & 1][0][m]), wo = as_f16x8(f1[t & 1][1][m]);
#pragma unroll
                for (int h = 0; h < TP; ++h) {
                    bcc[h][m] = MFMA_F16(wh, ah[t & 1][h], t == 0 ? b1[m >> 1][m & 1] : bcc[h][m], 0, 0, 0);
                    bcl[h][m] = MFMA_F16(wh, al[t & 1][h], t == 0 ? z4 : bcl[h][m], 0, 0, 0);
                    bcl[h][m] = MFMA_F16(wo, ah[t & 1][h], bcl[h][m], 0, 0, 0);
                }
            }
            if (t + 1 < KT1) split1(t + 1, (t + 1) & 1);
#if DRL_QC4_IGLP1
            if (t + 1 < KT1) {  // the next slice's split interleaved with this slice's MFMAs: 1 MFMA, 3 VALU
#pragma unroll
                for (int i = 0; i < 3 * TP * NT1; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                }
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts2 = __builtin_amdgcn_s_memtime();
#endif
        // ---- the output layer: tile h's split beside tile h - 1's MFMAs
        f32x4 qf[TP];
        f16x8 ah2[2][KT2], al2[2][KT2];
        auto split2 = [&](int h, int b) __attribute__((always_inline)) {
#pragma unroll
            for (int s2 = 0; s2 < KT2; ++s2) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * s2 + (j >> 2), i = j & 3;
                    v[j] = qc4_relu(bcc[h][m][i] + bcl[h][m][i] * kLo);  // (layer 1's bias: bcc's initial value)
                }
                qc4_split(v, ah2[b][s2], al2[b][s2], mx);
            }
        };
        split2(0, 0);
#pragma unroll
        for (int h = 0; h < TP; ++h) {
            f32x4 qc, ql;
#pragma unroll
            for (int t = 0; t < KT2; ++t) {
                const f16x8 wh = as_f16x8(f2h[t]), wo = as_f16x8(f2l[t]);
                qc = MFMA_F16(wh, ah2[h & 1][t], t == 0 ? z4 : qc, 0, 0, 0);
                ql = MFMA_F16(wh, al2[h & 1][t], t == 0 ? z4 : ql, 0, 0, 0);
                ql = MFMA_F16(wo, ah2[h & 1][t], ql, 0, 0, 0);
            }
            if (h + 1 < TP) split2(h + 1, (h + 1) & 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) qf[h][i] = (qc[i] + ql[i] * kLo) + bq[i];
        }
        // ---- epsilon-greedy act, one env per lane: lane (c, g) takes env c of tile g, whose Q rows 4g' + i
        // sit in lane (c, g') register i of qf[g]
        float q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int src = c + 16 * (i >> 2);
            float v = __shfl(qf[0][i & 3], src);
#pragma unroll
            for (int h = 1; h < TP; ++h) {
                const float u = __shfl(qf[h][i & 3], src);
                v = g == h ? u : v;
            }
            q[i] = v;
        }
        if (env < a.E) {
            int best = 0;
            float bv = q[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) {
                const bool b = i < a.n_actions && q[i] > bv;
                best = b ? i : best;
                bv = b ? q[i] : bv;
            }
            a.actions[env * a.action_stride] = explore >= 0 ? explore : best;
#ifndef DRL_QC_STAMPS
            if (a.q)
                for (int i = 0; i < a.n_actions; ++i) a.q[env * a.n_actions + i] = q[i];
#endif
        }
#ifdef DRL_QC_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts3 = __builtin_amdgcn_s_memtime();
        if (lane == 0 && a.q) {
            uint32_t* st = reinterpret_cast<uint32_t*>(a.q) + grp * 5;
            st[0] = (uint32_t)(ts1 - ts0);
            st[1] = (uint32_t)(ts2 - ts1);
            st[2] = (uint32_t)(ts3 - ts2);
            st[3] = (uint32_t)(ts0 - t_entry);
            st[4] = (uint32_t)(ts3 - t_entry);
            uint32_t* sl = reinterpret_cast<uint32_t*>(a.q) + ngroups * 5 + grp * KP;
            for (int t = 0; t < KP; ++t) sl[t] = slice_ts[t];
        }
#endif
        if (ngrp < gend) {
#pragma unroll
            for (int h = 0; h < TP; ++h)
#pragma unroll
                for (int i = 0; i < 4 * NV; ++i) cw[h][i] = ncw[h][i];
        }
    }
    bool bad = mx >= 0x477ff000u;  // 65520.0f (NaN cannot reach a split: see split_f16)
    bad |= lane == 0 && reinterpret_cast<const int32_t*>(a.packed + a.status_vec)[0] != 0;  // pack range flag
    if (__ballot(bad) && lane == 0 && a.err) atomicOr(a.err, DRL_ERR_QNET_RANGE);
    if (a.synth_n > 1) {  // as in drl_qnet_act_kernel (TP 16-env tiles per group)
        const uint32_t nd = (uint32_t)a.synth_n - 1u;
        const uint32_t per = (uint32_t)(TP * 16) * nd;
        for (int64_t gg = grp0; gg < gend; gg += gstride) {
            for (uint32_t k = (uint32_t)lane; k < per; k += 64u) {
                const uint32_t el = k / nd;
                const int64_t env = TP * 16 * gg + el;
                const uint64_t drone = 1u + (k - el * nd);
                if (env < a.E) {
                    const uint64_t ctr = (a.synth_step << 40) ^ ((uint64_t)(a.env_offset + env) << 8) ^ drone;
                    const uint64_t hh = qn_splitmix64(a.synth_seed ^ qn_splitmix64(ctr));
                    a.actions[env * a.action_stride + (int64_t)drone] = (int32_t)(((hh >> 32) * 5ull) >> 32);
                }
            }
        }
    }
}

// ------------------------------------------------------------ add_many ---
// Transition i of the batch goes to slot (cursor + i) % capacity; with more
// transitions than slots only the last `capacity` are written (what a
// sequential add() loop leaves; XLA's duplicate-index scatter in add_many
// leaves the order unspecified).
// Slot of the r-th landing row: (cursor + first + r) % capacity without a
// 64-bit division (r < capacity; base = (cursor + first) % capacity, host).
__device__ __forceinline__ int64_t ring_slot(const ReplayArgs& a, uint32_t r) {
    const int64_t s = a.base + (int64_t)r;
    return s >= a.capacity ? s - a.capacity : s;
}

// One thread per float2 of the rows that land (flattened [rows][obs_floats/2]:
// coalesced over rows, ring-buffer slots contiguous except at the wrap); the
// thread of column 0 also copies the row's action / reward / done.
__global__ void __launch_bounds__(256) drl_replay_add_kernel(ReplayArgs a, FastDiv dcols, uint32_t total) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= total) return;
    const uint32_t D2 = (uint32_t)a.obs_floats / 2u;
    const uint32_t r = __umulhi(k, dcols.m), col = k - r * D2;  // D2 >= 1; dcols.one handled by the host
    const int64_t i = a.first + r;
    const int64_t slot = ring_slot(a, r);
    const float2 o = reinterpret_cast<const float2*>(a.obs + i * a.obs_stride)[col];
    const float2 nx = reinterpret_cast<const float2*>(a.next_obs + i * a.next_obs_stride)[col];
    reinterpret_cast<float2*>(a.buf_obs + slot * a.obs_floats)[col] = o;
    reinterpret_cast<float2*>(a.buf_next_obs + slot * a.obs_floats)[col] = nx;
    if (col == 0) {
        a.buf_actions[slot] = a.actions[i * a.action_stride];
        a.buf_rewards[slot] = a.rewards[i * a.reward_stride];
        a.buf_dones[slot] = a.dones[i * a.done_stride];
    }
}

// The same with one thread per 16-B chunk, for rows that are whole 16-B vectors at 16-B aligned addresses (the
// 128-B policy-code rows): a quarter of the threads of the float2 form, whose launch was latency-bound (5 us for
// 10,000 code-row transitions in the C3 train loop, profiles/r04_final/loop_*).
__global__ void __launch_bounds__(256) drl_replay_add16_kernel(ReplayArgs a, FastDiv dcols, uint32_t total) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= total) return;
    const uint32_t D4 = (uint32_t)a.obs_floats / 4u;
    const uint32_t r = __umulhi(k, dcols.m), col = k - r * D4;  // D4 >= 2
    const int64_t i = a.first + r;
    const int64_t slot = ring_slot(a, r);
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const u4v o = reinterpret_cast<const u4v*>(a.obs + i * a.obs_stride)[col];
    const u4v nx = reinterpret_cast<const u4v*>(a.next_obs + i * a.next_obs_stride)[col];
    // the ring rows are read back only by a later sample: streaming (nt) stores keep them out of the caches the
    // next act and step read from
    __builtin_nontemporal_store(o, reinterpret_cast<u4v*>(a.buf_obs + slot * a.obs_floats) + col);
    __builtin_nontemporal_store(nx, reinterpret_cast<u4v*>(a.buf_next_obs + slot * a.obs_floats) + col);
    // the row's scalars from three different lanes (their loads are gathers: one each, in parallel)
    if (col == 1) a.buf_actions[slot] = a.actions[i * a.action_stride];
    if (col == 2 % D4) a.buf_rewards[slot] = a.rewards[i * a.reward_stride];
    if (col == 3 % D4) a.buf_dones[slot] = a.dones[i * a.done_stride];
}

__global__ void drl_replay_add_rows_kernel(ReplayArgs a) {  // fallback for huge batches: block per row
    const int64_t i = a.first + blockIdx.x;
    if (i >= a.n) return;
    const int64_t slot = ring_slot(a, blockIdx.x);
    const int D2 = a.obs_floats / 2;
    const float2* so = reinterpret_cast<const float2*>(a.obs + i * a.obs_stride);
    const float2* sn = reinterpret_cast<const float2*>(a.next_obs + i * a.next_obs_stride);
    float2* dobs = reinterpret_cast<float2*>(a.buf_obs + slot * a.obs_floats);
    float2* dnext = reinterpret_cast<float2*>(a.buf_next_obs + slot * a.obs_floats);
    for (int k = threadIdx.x; k < D2; k += blockDim.x) {
        dobs[k] = so[k];
        dnext[k] = sn[k];
    }
    if (threadIdx.x == 0) {
        a.buf_actions[slot] = a.actions[i * a.action_stride];
        a.buf_rewards[slot] = a.rewards[i * a.reward_stride];
        a.buf_dones[slot] = a.dones[i * a.done_stride];
    }
}

hipError_t launch_qnet_pack(const QnetPack& p, hipStream_t s) {
    const int64_t n = p.n_wfrag_elems + p.n_bias;
    hipLaunchKernelGGL(drl_qnet_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_qnet_act(const QnetArgs& a, int num_cus, hipStream_t s) {
    if (a.precision == DRL_QNET_F32) {
        constexpr int TP = QN_TILES_F32;
        const int64_t ng = ((a.E + 15) / 16 + TP - 1) / TP;
        int64_t nb = (ng + QN_WAVES - 1) / QN_WAVES;
        if (nb > num_cus) nb = num_cus;
        const dim3 grid((unsigned)nb), block(64 * QN_WAVES);
        const size_t lds = (size_t)a.lds_vec * 16;
#define QN_F32_LAUNCH(NT)                                                                     \
    if (a.lo0_lds) hipLaunchKernelGGL((drl_qnet_act_f32_kernel<NT, TP, true>), grid, block, lds, s, a); \
    else hipLaunchKernelGGL((drl_qnet_act_f32_kernel<NT, TP, false>), grid, block, lds, s, a)
        switch (a.nt[0]) {
            case 2: QN_F32_LAUNCH(2); break;
            case 4: QN_F32_LAUNCH(4); break;
            case 6: QN_F32_LAUNCH(6); break;
            case 8: QN_F32_LAUNCH(8); break;
            default: return hipErrorInvalidValue;
        }
#undef QN_F32_LAUNCH
        return hipGetLastError();
    }
    const int64_t ngroups = ((a.E + 15) / 16 + QN_TILES - 1) / QN_TILES;
    int64_t blocks = (ngroups + QN_WAVES - 1) / QN_WAVES;
    if (blocks > num_cus) blocks = num_cus;
    const dim3 grid((unsigned)blocks), block(64 * QN_WAVES);
    const size_t lds = (size_t)a.lds_vec * 16;
    switch (a.nt[0]) {
        case 2: hipLaunchKernelGGL(drl_qnet_act_kernel<2>, grid, block, lds, s, a); break;
        case 4: hipLaunchKernelGGL(drl_qnet_act_kernel<4>, grid, block, lds, s, a); break;
        case 6: hipLaunchKernelGGL(drl_qnet_act_kernel<6>, grid, block, lds, s, a); break;
        case 8: hipLaunchKernelGGL(drl_qnet_act_kernel<8>, grid, block, lds, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static bool blocks_ok(const QnetArgs& a) { return a.lds_vec == 2 * a.frag_lo_off[0]; }

hipError_t launch_qnet_act_code(const QnetArgs& a, int window, int num_cus, hipStream_t s) {
    static const int waves = [] {  // DRL_QN_CODE_WAVES: waves per workgroup (A/B knob)
        const char* e = getenv("DRL_QN_CODE_WAVES");
        const int w = e ? atoi(e) : QN_CODE_WAVES;
        return w >= 1 && w <= QN_CODE_MAXW ? w : QN_CODE_WAVES;
    }();
    const int64_t nt = (a.E + 15) / 16;
    int64_t nb = (nt + waves - 1) / waves;
    if (nb > num_cus) nb = num_cus;
    const dim3 grid((unsigned)nb), block(64 * waves);
    const size_t lds = (size_t)a.lds_vec * 16;
    int64_t nb2 = ((nt + 1) / 2 + QN_CODE2_WAVES - 1) / QN_CODE2_WAVES;  // (two tiles per wave)
    if (nb2 > num_cus) nb2 = num_cus;
    const dim3 grid2((unsigned)nb2), block2(64 * QN_CODE2_WAVES);
#define QN_CODE_LAUNCH(NT, W)                                                                                   \
    if (a.lo0_lds) hipLaunchKernelGGL((drl_qnet_act_code_kernel<NT, true, W, 0>), grid, block, lds, s, a);     \
    else hipLaunchKernelGGL((drl_qnet_act_code_kernel<NT, false, W, 0>), grid, block, lds, s, a)
    // DRL_QN_CODE=2: the two-tile kernel for the benchmark nets too (A/B knob, read per call so the parity
    // test can reach drl_qnet_act_code2_kernel: no packable net needs it at 32-bit code offsets)
    const char* v2e = getenv("DRL_QN_CODE");
    const bool v2 = v2e && v2e[0] == '2';
    const int64_t ng4 = (nt + 3) / 4;  // drl_qnet_act_code4_kernel: four tiles per wave, four waves per workgroup
    int64_t nb4 = (ng4 + QC4_WAVES - 1) / QC4_WAVES;
    if (nb4 > num_cus) nb4 = num_cus;
    const dim3 grid4((unsigned)nb4), block4(64 * QC4_WAVES);
    // drl_qnet_act_code4_kernel: the lo0_lds layout (layer 0's hi then lo fragments from offset 0), 128 units,
    // a window whose layer 0 fits the LDS (5x5, 7x7), 32-bit code offsets; drl_qnet_act_code2_kernel otherwise
    const bool v4ok = !v2 && a.lo0_lds && a.frag_off[0] == 0 && window <= 7 &&
                      a.frag_lo_off[0] == 8 * lay::code_kt(window) * 64 && blocks_ok(a) &&
                      a.E * (int64_t)lay::code_bytes(window) < (1ll << 31);
#define QN_CODE_SPEC(W)                                                                                         \
    if (v4ok && W <= 7) hipLaunchKernelGGL((drl_qnet_act_code4_kernel<8, (W <= 7 ? W : 7), 4>), grid4, block4, lds, s, a); \
    else if (a.lo0_lds) hipLaunchKernelGGL((drl_qnet_act_code2_kernel<8, true, W, 4>), grid2, block2, lds, s, a);   \
    else hipLaunchKernelGGL((drl_qnet_act_code2_kernel<8, false, W, 4>), grid2, block2, lds, s, a)
    const bool spec = a.n_hidden == 2 && a.nt[0] == 8 && a.nt[1] == 4;  // 128 -> 64 hidden
#define QN_CODE_W(W)                             \
    if (spec) { QN_CODE_SPEC(W); } else           \
    switch (a.nt[0]) {                            \
        case 2: QN_CODE_LAUNCH(2, W); break;      \
        case 4: QN_CODE_LAUNCH(4, W); break;      \
        case 6: QN_CODE_LAUNCH(6, W); break;      \
        case 8: QN_CODE_LAUNCH(8, W); break;      \
        default: return hipErrorInvalidValue;     \
    }
    switch (window) {
        case 5: QN_CODE_W(5) break;
        case 7: QN_CODE_W(7) break;
        case 9: QN_CODE_W(9) break;
        default: return hipErrorInvalidValue;
    }
#undef QN_CODE_W
#undef QN_CODE_SPEC
#undef QN_CODE_LAUNCH
    return hipGetLastError();
}

hipError_t launch_replay_add(const ReplayArgs& a, hipStream_t s) {
    const int64_t rows = a.n - a.first;
    if (rows <= 0) return hipSuccess;
    const uint64_t D2 = (uint64_t)a.obs_floats / 2;
    const uint64_t total = (uint64_t)rows * D2;
    const uint64_t D4 = (uint64_t)a.obs_floats / 4, total4 = (uint64_t)rows * D4;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    if (a.obs_floats % 4 == 0 && D4 >= 2 && a.obs_stride % 4 == 0 && a.next_obs_stride % 4 == 0 && al16(a.obs) &&
        al16(a.next_obs) && al16(a.buf_obs) && al16(a.buf_next_obs) && total4 * D4 < (1ull << 32)) {
        hipLaunchKernelGGL(drl_replay_add16_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, a,
                           make_fastdiv((uint32_t)D4), (uint32_t)total4);
    } else if (D2 >= 2 && total * D2 < (1ull << 32)) {  // multiply-shift row index exact (FastDiv bound)
        hipLaunchKernelGGL(drl_replay_add_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a,
                           make_fastdiv((uint32_t)D2), (uint32_t)total);
    } else {
        hipLaunchKernelGGL(drl_replay_add_rows_kernel, dim3((unsigned)rows), dim3(64), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace drl
