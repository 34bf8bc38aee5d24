// dronerl_qnet_api.cpp — C ABI of the DQN consumer (include/dronerl.h,
// drl_qnet_* / drl_replay_add; kernels in dronerl_qnet.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/dronerl.h"
#include "dronerl_internal.h"

extern "C" __attribute__((visibility("hidden"))) int drl_internal_fail(const char* msg);

namespace {

constexpr int kQnetLdsMax = 160 * 1024;

int fail(const char* m) { return drl_internal_fail(m); }

// Validate a description and lay the packed net out (see QnetLayout).
int qnet_layout(const drl_qnet_desc* d, drl::QnetLayout* L) {
    if (!d) return fail("qnet desc is NULL");
    if (d->in_features < 4 || d->in_features > 512 || (d->in_features & 1))
        return fail("in_features must be even and in [4, 512]");
    if (d->n_hidden < 1 || d->n_hidden > 3) return fail("n_hidden must be 1, 2 or 3");
    for (int i = 0; i < d->n_hidden; ++i)
        if (d->hidden[i] < 32 || d->hidden[i] > 128 || d->hidden[i] % 32)
            return fail("hidden widths must be multiples of 32 in [32, 128]");
    if (d->n_actions < 1 || d->n_actions > 8) return fail("n_actions must be in [1, 8]");
    if (d->precision != DRL_QNET_BF16 && d->precision != DRL_QNET_F32)
        return fail("precision must be DRL_QNET_BF16 or DRL_QNET_F32");
    int code_w = 0;
    if (d->input == DRL_QNET_INPUT_CODE) {
        for (int w = 5; w <= 9; w += 2)
            if (d->in_features == w * w * 6) code_w = w;
        if (!code_w) return fail("a policy-code net takes a 5x5, 7x7 or 9x9 window (in_features W*W*6)");
        if (d->precision != DRL_QNET_F32) return fail("a policy-code net runs DRL_QNET_F32");
    } else if (d->input != DRL_QNET_INPUT_OBS) {
        return fail("input must be DRL_QNET_INPUT_OBS or DRL_QNET_INPUT_CODE");
    }
    memset(L, 0, sizeof *L);
    L->code_w = code_w;
    L->precision = d->precision;
    L->n_layers = d->n_hidden + 1;
    int frag = 0, bias = 0;
    for (int l = 0; l < L->n_layers; ++l) {
        L->in[l] = l == 0 ? d->in_features : d->hidden[l - 1];
        L->out[l] = l < d->n_hidden ? d->hidden[l] : d->n_actions;
        L->nt[l] = (L->out[l] + 15) / 16;  // 16-row MFMA tiles
        // 32-wide K-slices; layer 0 padded to a multiple of the act kernel's slice ring
        constexpr int R = drl::lay::qn_ring;
        L->kt[l] = l == 0 ? (code_w ? drl::lay::code_kt(code_w) : ((d->in_features + 31) / 32 + R - 1) / R * R)
                          : L->in[l] / 32;
        L->frag_off[l] = frag * 64;
        L->frag_src[l] = frag * 64;
        L->bias_off[l] = bias;
        frag += L->nt[l] * L->kt[l];
        bias += 16 * L->nt[l];
    }
    L->frag_total = frag * 64;
    L->n_bias = bias;
    L->bias_vec = L->frag_total;
    L->lds_vec = L->frag_total + (bias + 3) / 4;
    if (d->precision == DRL_QNET_F32) {
        const int f0 = L->nt[0] * L->kt[0] * 64;
#ifndef DRL_QNET_LO0_LDS
#define DRL_QNET_LO0_LDS 1
#endif
        if (DRL_QNET_LO0_LDS && 2 * f0 * 16 <= kQnetLdsMax) {
            // layer 0's hi and lo fragments are the LDS image (160 KB at
            // 294->128); the later layers' fragments and the biases follow in
            // global memory (L2-resident, a few KB per 16-env tile)
            L->lo0_lds = 1;
            L->frag_lo_off[0] = f0;
            int pos = 2 * f0;
            L->lds_vec = pos;
            for (int l = 1; l < L->n_layers; ++l) {
                L->frag_off[l] = pos;
                pos += L->nt[l] * L->kt[l] * 64;
            }
            L->bias_vec = pos;
            pos += (bias + 3) / 4;
            for (int l = 1; l < L->n_layers; ++l) {
                L->frag_lo_off[l] = pos;
                pos += L->nt[l] * L->kt[l] * 64;
            }
            L->total_vec = pos;
        } else {
            // lo fragments: the hidden and output layers' after the biases (LDS
            // image), layer 0's after the image (read from global memory / L2)
            for (int l = 1; l < L->n_layers; ++l) {
                L->frag_lo_off[l] = L->lds_vec;
                L->lds_vec += L->nt[l] * L->kt[l] * 64;
            }
            L->frag_lo_off[0] = L->lds_vec;
            L->total_vec = L->lds_vec + f0;
        }
    } else {
        L->total_vec = L->lds_vec;
    }
    // a 16-B status vector ends the packed net: drl_qnet_pack ORs
    // DRL_ERR_QNET_RANGE into its first word when a weight (or a code net's
    // layer-0 bias, packed as a weight) is outside fp16's split range or not
    // finite, and the f32 act kernels report it through their err word
    L->status_vec = L->total_vec;
    L->total_vec += 1;
    if (L->lds_vec * 16 > kQnetLdsMax) return fail("the packed network does not fit the 160 KB LDS of a CU");
    return 0;
}

int hip_fail(hipError_t e, const char* what) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return fail(buf);
}

int num_cus() {
    static std::mutex mu;
    static std::vector<int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> g(mu);
    if ((int)cache.size() <= dev) cache.resize(dev + 1, 0);
    if (!cache[dev]) {
        int n = 0;
        cache[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cache[dev];
}


// drl::dqn_train_resident_capacity per (device, LDS bytes), queried once
static int dqn_resident_capacity(size_t lds) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<int, size_t>, int>> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    std::lock_guard<std::mutex> g(mu);
    for (const auto& c : cache)
        if (c.first.first == dev && c.first.second == lds) return c.second;
    const int cap = drl::dqn_train_resident_capacity(lds, num_cus());
    if (cap >= 0) cache.push_back({{dev, lds}, cap});
    return cap;
}

// The agent block of a learner (include/dronerl.h drl_dqn_layout), the scratch
// regions of drl::LearnArgs, and the gradient launch's LDS.
struct DqnPlan {
    drl_dqn_layout pub;
    int64_t sz0, smx, sd1, spx, sh[drl::QN_MAX_LAYERS], sd[drl::QN_MAX_LAYERS];  // float offsets in the scratch
    int in4, xs0, maxw, tiles0, ws_floats, region_a, prefetch;
    int tw[2][drl::QN_MAX_LAYERS], tb[2][drl::QN_MAX_LAYERS], tm[drl::QN_MAX_LAYERS], tv[drl::QN_MAX_LAYERS], tr;
    int twt[drl::QN_MAX_LAYERS];
    size_t lds;
};

static int64_t r4(int64_t v) { return (v + 3) / 4 * 4; }

// DqSeg::rm: i / row == umulhi(i, rm) exactly for i * row < 2^32 (drl::FastDiv's multiplier)
static uint32_t rm_of(int row) { return row > 1 ? drl::make_fastdiv((uint32_t)row).m : 0u; }

static int dqn_plan(const drl_qnet_desc* d, int32_t batch, const drl::QnetLayout& L, DqnPlan* P) {
    if (batch < 1 || batch > drl::DQN_MAX_BATCH) return fail("batch must be in [1, 64]");
    memset(P, 0, sizeof *P);
    drl_dqn_layout& o = P->pub;
    int64_t f = 0;
    for (int l = 0; l < L.n_layers; ++l) {
        o.weight_off[l] = f;
        f += r4((int64_t)L.in[l] * L.out[l]);
        o.bias_off[l] = f;
        f += r4(L.out[l]);
    }
    o.n_params = f;
    const int64_t set = f * 4;
    o.online_off = 0;
    o.target_off = set;
    o.m_off = 2 * set;
    o.v_off = 3 * set;
    o.counters_off = 4 * set;
    o.scratch_off = o.counters_off + (int64_t)sizeof(drl::DqnCounters);
    P->in4 = (int)r4(L.in[0]);
    int maxw = 0;
    for (int l = 0; l < L.n_layers; ++l) maxw = L.out[l] > maxw ? L.out[l] : maxw;
    P->maxw = (int)r4(maxw);
    int64_t sc = 0;
    P->sz0 = sc;  // granules: 8 B each
    sc += r4(2 * 2ll * batch * L.out[0]);
    P->smx = sc;
    sc += r4(2ll * batch);
    P->sd1 = sc;  // layer-1 delta granules
    sc += L.n_layers > 1 ? r4(2ll * batch * L.out[1]) : 0;
    P->spx = sc;  // the weights' packed-image elements (drl_dqn_init)
    sc += r4(f);
    for (int l = 0; l + 1 < L.n_layers; ++l) {
        P->sh[l] = sc;
        sc += r4((int64_t)batch * L.out[l]);
    }
    for (int l = 0; l < L.n_layers; ++l) {
        P->sd[l] = sc;
        sc += r4((int64_t)batch * L.out[l]);
    }
#ifdef DRL_DQN_STAMPS
    sc += 2048;  // 8 KB of stamps (tools/learn_stamps.py)
#endif
    o.bytes = o.scratch_off + sc * 4;
    P->tiles0 = (L.out[0] + drl::DQN_TILE - 1) / drl::DQN_TILE;
    if ((int64_t)L.in[0] * drl::DQN_TILE > (int64_t)drl::DQN_W0R * drl::DQN_THREADS)  // (in <= 512 by qnet_layout)
        return fail("internal: a layer-0 tile does not fit the learner's weight registers");
    o.grad_workgroups = 2 * P->tiles0 + 2;
    // region A: layer 0 (X, the weight tile and its biases, a code net's sampled rows), then the last
    // workgroup's two activation buffers of one net and the online net's ReLU masks (+ one layer's weights
    // with rows of in + 4 floats when the tail is not prefetched)
    int ws = 0;
    for (int l = 1; l < L.n_layers; ++l) ws = std::max(ws, L.out[l] * (L.in[l] + 4));
    P->ws_floats = ws;
    P->xs0 = L.in[0] + ((4 - L.in[0]) % 32 + 32) % 32;  // (= 4 mod 32: dq_mm1's 8 rows x 4 classes, 32 banks)
    const int rw = L.code_w ? drl::lay::code_bytes(L.code_w) / 4 : 0;
    // the layer-0 workgroups: X, the weight tile and its biases, a code net's sampled rows
    // (+ the tile's pre-activations Z; with a hidden layer, the online tile's slice of W_1 [out1][TILE + 1]
    // and the handed-over layer-1 deltas [B][out1], from which it forms its own layer-0 deltas)
    const int64_t w1s = L.n_layers > 1 ? (int64_t)L.out[1] * (drl::DQN_TILE + 1) + (int64_t)batch * L.out[1] : 0;
    int64_t a0 = (int64_t)batch * P->in4 + (int64_t)drl::DQN_TILE * P->xs0 + drl::DQN_TILE + (int64_t)batch * rw +
                 (int64_t)batch * drl::DQN_TILE + w1s;
    int64_t later = 0;  // a target layer-0 workgroup's update phase: D_l and H_{l-1} of the later layers
    for (int l = 1; l < L.n_layers; ++l) later += (int64_t)batch * (L.out[l] + L.in[l]);
    a0 = std::max(a0, later);
    // the tail workgroup: two activation buffers of one net, the online net's ReLU masks (+ one layer's weights
    // with rows of in + 4 floats when the tail does not hold them), then the tail
    const int64_t masks = r4((int64_t)(L.n_layers - 1) * batch * P->maxw) / 4;
    const int64_t a1p = 2ll * batch * P->maxw + masks, a1s = a1p + ws;
    // the prefetched tail: every bias of both nets, the online biases' moments, the sampled rows' action /
    // reward / done, then (when they fit) the later layers' weights of both nets
    int64_t t = 0;
    for (int n = 0; n < 2; ++n)
        for (int l = 0; l < L.n_layers; ++l) {
            P->tb[n][l] = (int)t;
            t += r4(L.out[l]);
        }
    for (int l = 0; l < L.n_layers; ++l) {
        P->tm[l] = (int)t;
        t += r4(L.out[l]);
        P->tv[l] = (int)t;
        t += r4(L.out[l]);
    }
    P->tr = (int)t;
    t += r4(3ll * batch);
    const int64_t t_small = t;
    for (int l = 1; l < L.n_layers; ++l) {  // (each tail holds its own net's weights: the same offsets)
        P->tw[0][l] = P->tw[1][l] = (int)t;
        t += (int64_t)L.out[l] * (L.in[l] + 2);  // (rows of in + 2 floats: dq_mm's bank pattern)
    }
    for (int l = 2; l < L.n_layers; ++l) {  // the online tail's W_l^T for the backward pass (layer 0's deltas:
        P->twt[l] = (int)t;                    // the layer-0 workgroups, from W_1's columns)
        t += r4((int64_t)L.in[l] * (L.out[l] + 2));
    }
    constexpr int64_t kMaxFloats = 150 * 1024 / 4;  // (+ ~7 KB of the kernel's own LDS arrays)
    P->prefetch = std::max(a0, a1p + t) <= kMaxFloats;
    if (!P->prefetch) t = t_small;
    P->region_a = (int)(P->prefetch ? a1p : a1s);
    P->lds = (size_t)std::max(a0, P->region_a + t) * 4;
    o.grad_lds_bytes = (int32_t)P->lds;
    if (P->lds > 150 * 1024) return fail("the learner's batch and widths do not fit the LDS of a CU");
    (void)d;
    return 0;
}

}  // namespace

extern "C" {

int drl_qnet_packed_bytes(const drl_qnet_desc* d, int64_t* bytes) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!bytes) return fail("bytes is NULL");
    *bytes = (int64_t)L.total_vec * 16;
    return 0;
}

// The pack kernel's arguments for net layout L (weights / biases: nullable
// source pointers; the learner's update kernel writes from its own sets).
static void fill_pack(const drl::QnetLayout& L, void* d_packed, const float* const* w, const float* const* b,
                      drl::QnetPack* p) {
    memset(p, 0, sizeof *p);
    p->n_layers = L.n_layers;
    for (int l = 0; l < L.n_layers; ++l) {
        p->frag_off[l] = L.frag_off[l];
        p->frag_src[l] = L.frag_src[l];
        p->kt[l] = L.kt[l];
        p->in[l] = L.in[l];
        p->out[l] = L.out[l];
        p->bias_off[l] = L.bias_off[l];
        p->w[l] = w ? w[l] : nullptr;
        p->b[l] = b ? b[l] : nullptr;
        p->frag_lo_off[l] = L.frag_lo_off[l];
    }
    p->precision = L.precision;
    p->code_w = L.code_w;
    p->status = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(d_packed) + (size_t)L.status_vec * 16);
    p->n_wfrag_elems = (int64_t)L.frag_total * 8;
    p->n_bias = L.n_bias;
    p->packed_w = static_cast<uint16_t*>(d_packed);
    p->packed_b = reinterpret_cast<float*>(static_cast<uint8_t*>(d_packed) + (size_t)L.bias_vec * 16);
}

int drl_qnet_pack(const drl_qnet_desc* d, const float* const* d_weights, const float* const* d_biases, void* d_packed,
                  hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!d_weights || !d_biases || !d_packed) return fail("weights/biases/packed must be non-NULL");
    if ((uintptr_t)d_packed % 16) return fail("packed buffer must be 16-byte aligned");
    for (int l = 0; l < L.n_layers; ++l)
        if (!d_weights[l] || !d_biases[l]) return fail("a weight or bias pointer is NULL");
    drl::QnetPack p;
    fill_pack(L, d_packed, d_weights, d_biases, &p);
    if (hipError_t e0 = hipMemsetAsync(p.status, 0, 16, stream); e0 != hipSuccess)
        return hip_fail(e0, "drl_qnet_pack status reset");
    hipError_t e = drl::launch_qnet_pack(p, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_qnet_pack launch");
}

static int qnet_act_impl(const drl_qnet_desc* d, const void* d_packed, const float* d_obs, int64_t num_envs,
                         int64_t obs_stride, float epsilon, const float* eps_ptr, uint64_t seed, uint64_t step, int64_t env_offset,
                         int32_t* d_actions, int64_t action_stride, float* d_q, int synth_n, uint64_t synth_seed,
                         uint64_t synth_step, int32_t* d_err, hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (L.code_w) return fail("a DRL_QNET_INPUT_CODE net acts through drl_qnet_act_code");
    if (num_envs < 0) return fail("num_envs < 0");
    if (num_envs == 0) return 0;
    if (!d_packed || !d_obs || !d_actions) return fail("packed/obs/actions must be non-NULL");
    if ((uintptr_t)d_packed % 16) return fail("packed buffer must be 16-byte aligned");
    if ((uintptr_t)d_obs % 8 || obs_stride % 2) return fail("obs rows must be 8-byte aligned (even obs_stride)");
    if (obs_stride < d->in_features) return fail("obs_stride < in_features");
    if (num_envs * obs_stride * 4 >= ((int64_t)1 << 32)) return fail("obs larger than 4 GiB (32-bit row offsets)");
    if (action_stride < 1) return fail("action_stride must be >= 1");
    drl::QnetArgs a;
    memset(&a, 0, sizeof a);
    a.in_features = d->in_features;
    a.kt0 = L.kt[0];
    a.n_hidden = d->n_hidden;
    a.n_actions = d->n_actions;
    for (int l = 0; l < L.n_layers; ++l) {
        a.nt[l] = L.nt[l];
        a.frag_off[l] = L.frag_off[l];
        a.bias_off[l] = L.bias_off[l];
        a.frag_lo_off[l] = L.frag_lo_off[l];
    }
    a.precision = L.precision;
    a.frag_total = L.frag_total;
    a.bias_vec = L.bias_vec;
    a.lo0_lds = L.lo0_lds;
    a.lds_vec = L.lds_vec;
    a.n_bias = L.n_bias;
    a.status_vec = L.status_vec;
    a.packed = static_cast<const uint4*>(d_packed);
    a.obs = d_obs;
    a.obs_stride = obs_stride;
    a.E = num_envs;
    a.epsilon = epsilon;
    a.eps_ptr = eps_ptr;
    a.seed = seed;
    a.step = step;
    a.env_offset = env_offset;
    a.actions = d_actions;
    a.action_stride = action_stride;
    a.q = d_q;
    a.synth_n = synth_n;
    a.synth_seed = synth_seed;
    a.synth_step = synth_step;
    a.err = d_err;
    hipError_t e = drl::launch_qnet_act(a, num_cus(), stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_qnet_act launch");
}

int drl_qnet_act(const drl_qnet_desc* d, const void* d_packed, const float* d_obs, int64_t num_envs,
                 int64_t obs_stride, float epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                 int32_t* d_actions, int64_t action_stride, float* d_q, int32_t* d_err, hipStream_t stream) {
    return qnet_act_impl(d, d_packed, d_obs, num_envs, obs_stride, epsilon, nullptr, seed, step, env_offset, d_actions,
                         action_stride, d_q, 0, 0, 0, d_err, stream);
}

int drl_qnet_act_synth(const drl_qnet_desc* d, const void* d_packed, const float* d_obs, int64_t num_envs,
                       int64_t obs_stride, float epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                       int32_t* d_actions, int32_t n_drones, uint64_t synth_seed, uint64_t synth_step, float* d_q,
                       int32_t* d_err, hipStream_t stream) {
    if (n_drones < 1 || n_drones > 255) return fail("n_drones must be in [1, 255]");
    return qnet_act_impl(d, d_packed, d_obs, num_envs, obs_stride, epsilon, nullptr, seed, step, env_offset, d_actions,
                         n_drones, d_q, n_drones, synth_seed, synth_step, d_err, stream);
}

static int qnet_act_code_impl(const drl_qnet_desc* d, const void* d_packed, const void* d_code, int64_t num_envs,
                              float epsilon, const float* eps_ptr, uint64_t seed, uint64_t step, int64_t env_offset,
                              int32_t* d_actions, int64_t action_stride, int32_t synth_n, uint64_t synth_seed,
                              uint64_t synth_step, float* d_q, int32_t* d_err, hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!L.code_w) return fail("drl_qnet_act_code needs a DRL_QNET_INPUT_CODE net");
    if (num_envs < 0) return fail("num_envs < 0");
    if (num_envs == 0) return 0;
    if (!d_packed || !d_code || !d_actions) return fail("packed/code/actions must be non-NULL");
    if ((uintptr_t)d_packed % 16 || (uintptr_t)d_code % 16) return fail("packed and code must be 16-byte aligned");
    if (action_stride < 1) return fail("action_stride must be >= 1");
    if (synth_n > 1 && action_stride < synth_n) return fail("action_stride must be >= synth_n");
    if (synth_n > DRL_MAX_DRONES) return fail("synth_n must be <= DRL_MAX_DRONES (64)");
    drl::QnetArgs a;
    memset(&a, 0, sizeof a);
    a.in_features = d->in_features;
    a.kt0 = L.kt[0];
    a.n_hidden = d->n_hidden;
    a.n_actions = d->n_actions;
    for (int l = 0; l < L.n_layers; ++l) {
        a.nt[l] = L.nt[l];
        a.frag_off[l] = L.frag_off[l];
        a.bias_off[l] = L.bias_off[l];
        a.frag_lo_off[l] = L.frag_lo_off[l];
    }
    a.precision = L.precision;
    a.frag_total = L.frag_total;
    a.bias_vec = L.bias_vec;
    a.lo0_lds = L.lo0_lds;
    a.lds_vec = L.lds_vec;
    a.n_bias = L.n_bias;
    a.status_vec = L.status_vec;
    a.packed = static_cast<const uint4*>(d_packed);
    a.obs = static_cast<const float*>(d_code);
    a.E = num_envs;
    a.epsilon = epsilon;
    a.eps_ptr = eps_ptr;
    a.seed = seed;
    a.step = step;
    a.env_offset = env_offset;
    a.actions = d_actions;
    a.action_stride = action_stride;
    a.q = d_q;
    a.synth_n = synth_n > 1 ? synth_n : 0;
    a.synth_seed = synth_seed;
    a.synth_step = synth_step;
    a.err = d_err;
    a.total_bytes = L.total_vec * 16;
    hipError_t e = drl::launch_qnet_act_code(a, L.code_w, num_cus(), stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_qnet_act_code launch");
}

int drl_qnet_act_code(const drl_qnet_desc* d, const void* d_packed, const void* d_code, int64_t num_envs,
                      float epsilon, uint64_t seed, uint64_t step, int64_t env_offset, int32_t* d_actions,
                      int64_t action_stride, int32_t synth_n, uint64_t synth_seed, uint64_t synth_step, float* d_q,
                      int32_t* d_err, hipStream_t stream) {
    return qnet_act_code_impl(d, d_packed, d_code, num_envs, epsilon, nullptr, seed, step, env_offset, d_actions,
                              action_stride, synth_n, synth_seed, synth_step, d_q, d_err, stream);
}

int drl_qnet_act_eps(const drl_qnet_desc* d, const void* d_packed, const void* d_input, int64_t num_envs,
                     int64_t obs_stride, const float* d_epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                     int32_t* d_actions, int64_t action_stride, int32_t synth_n, uint64_t synth_seed,
                     uint64_t synth_step, float* d_q, int32_t* d_err, hipStream_t stream) {
    if (!d_epsilon) return fail("d_epsilon is NULL");
    if ((uintptr_t)d_epsilon % 4) return fail("d_epsilon must be 4-byte aligned");
    if (!d || d->input != DRL_QNET_INPUT_CODE) {
        if (synth_n > 1) {
            if (synth_n > 255) return fail("n_drones must be in [1, 255]");
            if (action_stride < synth_n) return fail("action_stride must be >= synth_n");
        }
        return qnet_act_impl(d, d_packed, static_cast<const float*>(d_input), num_envs, obs_stride, 0.0f, d_epsilon,
                             seed, step, env_offset, d_actions, action_stride, d_q, synth_n > 1 ? synth_n : 0,
                             synth_seed, synth_step, d_err, stream);
    }
    return qnet_act_code_impl(d, d_packed, d_input, num_envs, 0.0f, d_epsilon, seed, step, env_offset, d_actions,
                              action_stride, synth_n, synth_seed, synth_step, d_q, d_err, stream);
}

int drl_replay_add(const drl_replay* r, int64_t cursor, int64_t n, const float* d_obs, int64_t obs_stride,
                   const float* d_next_obs, int64_t next_obs_stride, const int32_t* d_actions, int64_t action_stride,
                   const float* d_rewards, int64_t reward_stride, const uint8_t* d_dones, int64_t done_stride,
                   hipStream_t stream) {
    if (!r) return fail("replay is NULL");
    if (r->capacity < 1 || r->obs_floats < 2 || (r->obs_floats & 1))
        return fail("replay capacity must be >= 1 and obs_floats even");
    if (!r->obs || !r->next_obs || !r->actions || !r->rewards || !r->dones) return fail("replay buffers are NULL");
    if (n < 0 || cursor < 0) return fail("n and cursor must be >= 0");
    if (n == 0) return 0;
    if (!d_obs || !d_next_obs || !d_actions || !d_rewards || !d_dones) return fail("batch pointers are NULL");
    if ((uintptr_t)d_obs % 8 || (uintptr_t)d_next_obs % 8 || (uintptr_t)r->obs % 8 || (uintptr_t)r->next_obs % 8 ||
        obs_stride % 2 || next_obs_stride % 2)
        return fail("observation rows must be 8-byte aligned");
    if (obs_stride < r->obs_floats || next_obs_stride < r->obs_floats)
        return fail("obs_stride / next_obs_stride < obs_floats");
    if (action_stride < 1 || reward_stride < 1 || done_stride < 1) return fail("action/reward/done strides must be >= 1");
    drl::ReplayArgs a;
    memset(&a, 0, sizeof a);
    a.n = n;
    a.first = n > r->capacity ? n - r->capacity : 0;  // earlier ones would be overwritten in the same call
    a.cursor = cursor % r->capacity;
    a.capacity = r->capacity;
    a.base = (a.cursor + a.first % r->capacity) % r->capacity;
    a.obs_floats = r->obs_floats;
    a.obs = d_obs;
    a.obs_stride = obs_stride;
    a.next_obs = d_next_obs;
    a.next_obs_stride = next_obs_stride;
    a.actions = d_actions;
    a.action_stride = action_stride;
    a.rewards = d_rewards;
    a.reward_stride = reward_stride;
    a.dones = d_dones;
    a.done_stride = done_stride;
    a.buf_obs = r->obs;
    a.buf_next_obs = r->next_obs;
    a.buf_actions = r->actions;
    a.buf_rewards = r->rewards;
    a.buf_dones = r->dones;
    hipError_t e = drl::launch_replay_add(a, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_replay_add launch");
}

int drl_dqn_layout_query(const drl_qnet_desc* d, int32_t batch, drl_dqn_layout* layout) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!layout) return fail("layout is NULL");
    DqnPlan P;
    if (dqn_plan(d, batch, L, &P)) return -1;
    *layout = P.pub;
    return 0;
}

int drl_dqn_init(const drl_qnet_desc* d, int32_t batch, void* d_agent, float epsilon_start, hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    DqnPlan P;
    if (dqn_plan(d, batch, L, &P)) return -1;
    if (!d_agent || (uintptr_t)d_agent % 16) return fail("the agent block must be a 16-byte aligned device pointer");
    uint8_t* base = static_cast<uint8_t*>(d_agent);
    const size_t set = (size_t)P.pub.n_params * 4;
    if (hipError_t e = hipMemsetAsync(base + P.pub.m_off, 0, 2 * set, stream); e != hipSuccess)
        return hip_fail(e, "drl_dqn_init moments");
    // the whole scratch: the hand-off granules' tags must not match a later epoch (a block from hipMalloc,
    // or one that has trained already)
    if (hipError_t e = hipMemsetAsync(base + P.pub.scratch_off, 0, (size_t)(P.pub.bytes - P.pub.scratch_off), stream);
        e != hipSuccess)
        return hip_fail(e, "drl_dqn_init scratch");
    // each weight's element in the act kernels' packed image (qnet_pack_elem, once: the learner reads it)
    std::vector<uint32_t> px((size_t)P.pub.n_params, 0u);
    for (int l = 0; l < L.n_layers; ++l)
        for (int row = 0; row < L.out[l]; ++row)
            for (int k = 0; k < L.in[l]; ++k) {
                const int64_t pe = drl::qnet_pack_elem(l, row, k, L.kt[l], L.code_w);
                const bool scale = l == 0 && L.code_w > 0 && k % 6 == 4;
                px[(size_t)(P.pub.weight_off[l] + (int64_t)row * L.in[l] + k)] = (uint32_t)pe | (scale ? 0x80000000u : 0u);
            }
    if (hipError_t e = hipMemcpyAsync(base + P.pub.scratch_off + P.spx * 4, px.data(), px.size() * 4,
                                      hipMemcpyHostToDevice, stream); e != hipSuccess)
        return hip_fail(e, "drl_dqn_init pack index");
    if (hipError_t e = hipStreamSynchronize(stream); e != hipSuccess)  // (px is a host temporary)
        return hip_fail(e, "drl_dqn_init pack index");
    hipError_t e = drl::launch_dqn_init(base + P.pub.counters_off, epsilon_start, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_dqn_init launch");
}

static int dqn_train_impl(const drl_qnet_desc* d, const drl_dqn_hparams* h, void* d_agent, void* d_packed,
                          const drl_replay* r, int64_t size, const drl_replay_batch* fresh, hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!h) return fail("hparams is NULL");
    DqnPlan P;
    if (dqn_plan(d, h->batch, L, &P)) return -1;
    if (h->target_update_interval < 1 || h->epsilon_decay_every < 1)
        return fail("target_update_interval and epsilon_decay_every must be >= 1");
    if (!(h->beta1 >= 0.0 && h->beta1 < 1.0 && h->beta2 >= 0.0 && h->beta2 < 1.0))
        return fail("beta1 and beta2 must be in [0, 1)");
    if (!d_agent || (uintptr_t)d_agent % 16) return fail("the agent block must be a 16-byte aligned device pointer");
    if (!d_packed || (uintptr_t)d_packed % 16) return fail("packed buffer must be a 16-byte aligned device pointer");
    if (!r || !r->obs || !r->next_obs || !r->actions || !r->rewards || !r->dones) return fail("replay buffers are NULL");
    if (r->capacity < 1 || r->capacity >= ((int64_t)1 << 31)) return fail("replay capacity must be in [1, 2^31)");
    if (size < 0 || size > r->capacity) return fail("size must be in [0, capacity]");
    if (L.code_w) {
        if ((int64_t)r->obs_floats * 4 != drl::lay::code_bytes(L.code_w))
            return fail("a DRL_QNET_INPUT_CODE net's replay rows are policy codes (drl_policy_code_bytes / 4 words)");
    } else if (r->obs_floats < d->in_features) {
        return fail("replay obs_floats < in_features");
    }
    if ((uintptr_t)r->obs % 4 || (uintptr_t)r->next_obs % 4) return fail("replay rows must be 4-byte aligned");
    if (size >= h->batch) {  // the workgroups poll each other's hand-offs: all of them must fit at once
        const int cap = dqn_resident_capacity(P.lds);
        if (cap < 0) return fail("drl_dqn_train: the occupancy query failed");
        if (cap < P.pub.grad_workgroups) {
            char buf[160];
            snprintf(buf, sizeof buf, "drl_dqn_train needs %d co-resident workgroups (%zu B of LDS each); "
                     "this device holds %d", P.pub.grad_workgroups, P.lds, cap);
            return fail(buf);
        }
    }
    uint8_t* base = static_cast<uint8_t*>(d_agent);
    drl::LearnArgs a;
    memset(&a, 0, sizeof a);
    a.spin_word = drl::DQN_SPIN_WORD;
    a.spin_granule = drl::DQN_SPIN_GRANULE;
    if (const char* v = getenv("DRL_DQN_DEBUG_DROP_HANDOFF"); v && v[0] == '1') {
        // (diagnostic, tests only: the target side's layer-0 workgroups then give up after a short wait)
        a.drop_handoff = 1;
        a.spin_word = 1u << 12;
        a.spin_granule = 1u << 12;
    }
    a.n_layers = L.n_layers;
    a.batch = h->batch;
    a.code_w = L.code_w;
    a.trained = size >= h->batch;  // buffers.py:92-93 can_sample
    a.tiles0 = P.tiles0;
    a.nblk0 = 2 * P.tiles0;
    a.maxw = P.maxw;
    a.in4 = P.in4;
    a.xs0 = P.xs0;
    a.rm_in = rm_of(L.in[0]);
    a.rm_rw = rm_of((int)r->obs_floats);
    a.ws_floats = P.ws_floats;
    a.region_a = P.region_a;
    a.prefetch = P.prefetch;
    a.tr = P.tr;
    for (int l = 0; l < L.n_layers; ++l) {
        a.tw[0][l] = P.tw[0][l];
        a.tw[1][l] = P.tw[1][l];
        a.twt[l] = P.twt[l];
        a.tb[0][l] = P.tb[0][l];
        a.tb[1][l] = P.tb[1][l];
        a.tm[l] = P.tm[l];
        a.tv[l] = P.tv[l];
    }
    for (int l = 0; l < L.n_layers; ++l) {
        a.in[l] = L.in[l];
        a.out[l] = L.out[l];
        a.woff[l] = P.pub.weight_off[l];
        a.boff[l] = P.pub.bias_off[l];
        a.n_params = P.pub.n_params;
    }
    a.online = reinterpret_cast<float*>(base + P.pub.online_off);
    a.target = reinterpret_cast<float*>(base + P.pub.target_off);
    a.adam_m = reinterpret_cast<float*>(base + P.pub.m_off);
    a.adam_v = reinterpret_cast<float*>(base + P.pub.v_off);
    a.ctr = reinterpret_cast<drl::DqnCounters*>(base + P.pub.counters_off);
    float* sc = reinterpret_cast<float*>(base + P.pub.scratch_off);
    a.gz0 = reinterpret_cast<uint64_t*>(sc + P.sz0);
    a.gmx = reinterpret_cast<uint64_t*>(sc + P.smx);
    a.gd1 = reinterpret_cast<uint64_t*>(sc + P.sd1);
    a.pidx = reinterpret_cast<const uint32_t*>(sc + P.spx);
    for (int l = 0; l < L.n_layers; ++l) {
        a.sh[l] = l + 1 < L.n_layers ? sc + P.sh[l] : nullptr;
        a.sd[l] = sc + P.sd[l];
    }
    a.r_obs = reinterpret_cast<const uint32_t*>(r->obs);
    a.r_next = reinterpret_cast<const uint32_t*>(r->next_obs);
    a.row_words = r->obs_floats;
    a.r_act = r->actions;
    a.r_rew = r->rewards;
    a.r_done = r->dones;
    a.size = size;
    a.capacity = r->capacity;
    a.seed = h->sample_seed;
    if (fresh && fresh->n > 0) {
        if (!fresh->obs || !fresh->next_obs || !fresh->actions || !fresh->rewards || !fresh->dones)
            return fail("fresh batch pointers are NULL");
        if (fresh->cursor < 0 || fresh->obs_stride < r->obs_floats || fresh->next_obs_stride < r->obs_floats ||
            fresh->action_stride < 1 || fresh->reward_stride < 1 || fresh->done_stride < 1)
            return fail("fresh batch: bad cursor or strides");
        if ((uintptr_t)fresh->obs % 4 || (uintptr_t)fresh->next_obs % 4) return fail("fresh rows must be 4-byte aligned");
        const int64_t first = fresh->n > r->capacity ? fresh->n - r->capacity : 0;
        a.fresh = 1;
        a.f_first = first;
        a.f_rows = fresh->n - first;
        a.f_base = (fresh->cursor % r->capacity + first % r->capacity) % r->capacity;
        a.f_obs = static_cast<const uint32_t*>(fresh->obs);
        a.f_next = static_cast<const uint32_t*>(fresh->next_obs);
        a.f_act = fresh->actions;
        a.f_rew = fresh->rewards;
        a.f_done = fresh->dones;
        a.f_obs_stride = fresh->obs_stride;
        a.f_next_stride = fresh->next_obs_stride;
        a.f_act_stride = fresh->action_stride;
        a.f_rew_stride = fresh->reward_stride;
        a.f_done_stride = fresh->done_stride;
    }
    // the python floats as jax's weak typing rounds them into f32 arithmetic
    a.gamma = (float)h->gamma;
    a.b1 = (float)h->beta1;
    a.b2 = (float)h->beta2;
    a.c1 = (float)(1.0 - h->beta1);
    a.c2 = (float)(1.0 - h->beta2);
    a.adam_eps = (float)h->adam_eps;
    a.neg_lr = (float)(-h->learning_rate);
    a.tau = (float)h->tau;
    a.one_minus_tau = (float)(1.0 - h->tau);
    a.eps_decay = (float)h->epsilon_decay;
    a.eps_end = (float)h->epsilon_end;
    a.inv_batch = 1.0f / (float)h->batch;
    a.b1d = h->beta1;
    a.b2d = h->beta2;
    a.target_every = h->target_update_interval;
    a.eps_every = h->epsilon_decay_every;
    {  // the tails' segments (drl::DqSeg): the online tail's, then the target tail's; the later layers'
       // weights only when they fit (a.prefetch)
        int ns = 0;
        const float* sets[2] = {a.online, a.target};
        auto seg = [&](const void* src, int n, int dst, int row, int pad, int kind) {
            a.tail[ns++] = drl::DqSeg{src, n, P.region_a + dst, row, pad, kind, rm_of(row), 0};
        };
        for (int n = 0; n < 2; ++n) {
            const int first = ns;
            if (a.prefetch)
                for (int l = 1; l < L.n_layers; ++l)
                    seg(sets[n] + P.pub.weight_off[l], L.in[l] * L.out[l] / 2, P.tw[n][l], L.in[l] / 2, 1, 5);
            if (n == 0) {
                // A (before the forward pass): the weights, the online biases of the later layers, the sampled
                // rows' action, reward, done (tables 2-4); C (behind the hand-off, for the bias updates): layer
                // 0's bias, the target biases, the moments.  (B, the rows behind the forward pass, measured
                // slower: their round trip then lands between the forward pass and the TD error)
                for (int l = 1; l < L.n_layers; ++l) seg(sets[0] + P.pub.bias_off[l], L.out[l], P.tb[0][l], 1, 0, 0);
                seg(nullptr, h->batch, P.tr, 1, 0, 1);
                a.tail[ns - 1].tbl = 2;
                seg(nullptr, h->batch, P.tr + h->batch, 1, 0, 1);
                a.tail[ns - 1].tbl = 3;
                seg(nullptr, h->batch, P.tr + 2 * h->batch, 1, 0, 2);
                a.tail[ns - 1].tbl = 4;
                a.ntail_a = ns - first;
                a.ntail_b = 0;
                seg(sets[0] + P.pub.bias_off[0], L.out[0], P.tb[0][0], 1, 0, 0);
                for (int l = 0; l < L.n_layers; ++l) seg(sets[1] + P.pub.bias_off[l], L.out[l], P.tb[1][l], 1, 0, 0);
                for (int l = 0; l < L.n_layers; ++l) {
                    seg(a.adam_m + P.pub.bias_off[l], L.out[l], P.tm[l], 1, 0, 0);
                    seg(a.adam_v + P.pub.bias_off[l], L.out[l], P.tv[l], 1, 0, 0);
                }
            } else {
                for (int l = 1; l < L.n_layers; ++l) seg(sets[1] + P.pub.bias_off[l], L.out[l], P.tb[1][l], 1, 0, 0);
            }
            a.ntail_of[n] = ns - first;
        }
        a.ntail = ns;
        a.tail_start[0] = 0;
        for (int g = 0; g < ns; ++g) a.tail_start[g + 1] = a.tail_start[g] + a.tail[g].n;
    }
    fill_pack(L, d_packed, nullptr, nullptr, &a.pack);
#ifdef DRL_DQN_STAMPS
    a.stamps = reinterpret_cast<uint64_t*>(base + P.pub.bytes - 8192);  // 16 per workgroup (<= 64)
#endif
    a.wstart[0] = 0;
    for (int l = 0; l < L.n_layers; ++l) a.wstart[l + 1] = a.wstart[l] + (int64_t)L.in[l] * L.out[l];
    hipError_t e = drl::launch_dqn_train(a, P.lds, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_dqn_train launch");
}

int drl_dqn_train(const drl_qnet_desc* d, const drl_dqn_hparams* h, void* d_agent, void* d_packed, const drl_replay* r,
                  int64_t size, hipStream_t stream) {
    return dqn_train_impl(d, h, d_agent, d_packed, r, size, nullptr, stream);
}

int drl_dqn_sample_rows(const drl_qnet_desc* d, const drl_dqn_hparams* h, const void* d_agent, int64_t size,
                        int64_t* d_slots, hipStream_t stream) {
    drl::QnetLayout L;
    if (qnet_layout(d, &L)) return -1;
    if (!h) return fail("hparams is NULL");
    DqnPlan P;
    if (dqn_plan(d, h->batch, L, &P)) return -1;
    if (!d_agent || (uintptr_t)d_agent % 16) return fail("the agent block must be a 16-byte aligned device pointer");
    if (!d_slots || (uintptr_t)d_slots % 8) return fail("d_slots must be an 8-byte aligned device pointer");
    if (size < 1) return fail("size must be >= 1 (buffers.py can_sample: nothing is drawn from an empty ring)");
    hipError_t e = drl::launch_dqn_sample(static_cast<const uint8_t*>(d_agent) + P.pub.counters_off, h->sample_seed,
                                          h->batch, size, d_slots, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_dqn_sample_rows launch");
}

int drl_dqn_train_fresh(const drl_qnet_desc* d, const drl_dqn_hparams* h, void* d_agent, void* d_packed,
                        const drl_replay* r, int64_t size, const drl_replay_batch* fresh, hipStream_t stream) {
    if (!fresh) return fail("fresh batch is NULL");
    return dqn_train_impl(d, h, d_agent, d_packed, r, size, fresh, stream);
}

}  // extern "C"
