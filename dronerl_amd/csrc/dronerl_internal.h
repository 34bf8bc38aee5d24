// Internal kernel argument blocks shared by dronerl_kernels.hip and dronerl_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dronerl.h"

namespace drl {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MT_WORDS = DRL_MT_WORDS;
constexpr int MT_ALT = DRL_MT_BLOCK1;  // word offset of MT block 1 in an env's row
constexpr int MT_RING = DRL_MT_RING;   // word offset of the respawn-candidate ring
constexpr int CAND_Q = DRL_CAND_SLOTS; // ring entries (power of two)
constexpr int MT_RING_END = DRL_MT_RING_END;  // word: stream position after the ring's last entry
static_assert((CAND_Q & (CAND_Q - 1)) == 0 && CAND_Q <= 512, "ring size");
static_assert(MT_RING_END < MT_WORDS && MT_RING + CAND_Q <= MT_RING_END && MT_WORDS % 16 == 0, "MT row layout");

// mt_index word (include/dronerl.h): index | par << 10 | head << 11 | count << 20
__host__ __device__ constexpr int mi_idx(uint32_t w) { return (int)(w & 0x3ffu); }
__host__ __device__ constexpr int mi_par(uint32_t w) { return (int)((w >> 10) & 1u); }
__host__ __device__ constexpr int mi_head(uint32_t w) { return (int)((w >> 11) & (uint32_t)(CAND_Q - 1)); }
__host__ __device__ constexpr int mi_cnt(uint32_t w) {
    return (int)((w >> 20) & 0x3ffu) < CAND_Q ? (int)((w >> 20) & 0x3ffu) : CAND_Q;
}
__host__ __device__ constexpr uint32_t mi_pack(int idx, int par, int head, int cnt) {
    return (uint32_t)idx | ((uint32_t)par << 10) | ((uint32_t)head << 11) | ((uint32_t)cnt << 20);
}
// candidate ring entry: cell | MT index after the pair << 16 | that index's block << 26
__host__ __device__ constexpr int ce_cell(uint32_t e) { return (int)(e & 0x3fffu); }
__host__ __device__ constexpr int ce_idx(uint32_t e) { return (int)((e >> 16) & 0x3ffu); }
__host__ __device__ constexpr int ce_par(uint32_t e) { return (int)((e >> 26) & 1u); }
__host__ __device__ constexpr uint32_t ce_pack(int cell, int idx, int par) {
    return (uint32_t)cell | ((uint32_t)idx << 16) | ((uint32_t)par << 26);
}
// ring entries each drl_step lane holds (P lanes per env: P * step_cq(P) candidates per step
// without a second memory round trip; more come from the stream itself)
// (DRL_CQ_NARROW: the count at P <= 16, a tuning knob for tools/variants.py builds)
#ifndef DRL_CQ_NARROW
#define DRL_CQ_NARROW 2
#endif
constexpr int step_cq(int P) { return P <= 16 ? DRL_CQ_NARROW : 1; }
// DRL_DPP8: P = 8 / 16 claim and crash-order scans by DPP lane swaps instead of ds_bpermute
#ifndef DRL_DPP8
#define DRL_DPP8 1
#endif
// dry-ring respawn rounds: D draws per lane (D*P MT outputs per round)
// (tuning knobs for tools/ab.py builds: DRL_DRAWS_P<P> overrides one width)
#ifndef DRL_DRAWS_P8
#define DRL_DRAWS_P8 2
#endif
#ifndef DRL_DRAWS_P16
#define DRL_DRAWS_P16 2
#endif
#ifndef DRL_DRAWS_P32
#define DRL_DRAWS_P32 1
#endif
constexpr int step_draws(int P) {
    return P == 8 ? DRL_DRAWS_P8 : P == 16 ? DRL_DRAWS_P16 : P == 32 ? DRL_DRAWS_P32 : 1;
}
// drl_rollout (several steps per launch, state on chip) runs at P >= 16, and
// at P = 8 without observations; otherwise narrower groups roll out as
// drl_step launches.  At C3 (P = 8) the on-chip kernel (85-100 VGPRs, 4-5
// waves per SIMD instead of the step kernel's 8) measured 12.1-12.2 us/step
// without obs against 13.7-13.8 for step launches, and 26.2 against 22.7-22.8
// with obs, whose stores want the step kernel's occupancy
// (profiles/r02_rollout_p8/).
constexpr int kRolloutMinLanes = 16;
constexpr int kRolloutNoObsMinLanes = 8;
// drl_rollout takes the rings' entries at group widths P <= DRL_ROLL_RING_MAXP
// and discards them at wider groups, drawing every respawn from the stream
// (the round-1 rollout's registers: one more wave per SIMD at C5).  Measured
// (profiles/r02_rollout_ring_ab/): C4 (P = 16) 27.95 vs 29.2 us/step with
// the entries, C5 (P = 32) 119.0 vs 134.2 without.  DRL_ROLL_RING=0 discards
// them at every width.
#ifndef DRL_ROLL_RING
#define DRL_ROLL_RING 1
#endif
#ifndef DRL_ROLL_RING_MAXP
#define DRL_ROLL_RING_MAXP 16
#endif
constexpr int OBS_U = 1;        // observation cells per lane per pass (stage: OBS_U*1536 B per wave)

// Per-env LDS layout of drl_step (WaveLds in dronerl_kernels.hip).  Shared by
// the host (launch sizes) and by the compile-time-geometry kernel instances.
namespace lay {
constexpr int r16(int v) { return (v + 15) / 16 * 16; }
constexpr int np(int n_drones) { return (n_drones + 7) / 8 * 8; }             // posidx entries
// ground: packed in HBM, one nibble per cell (cell 2i in the low nibble of
// byte i, 2i + 1 in the high one; ABI 8), unpacked to a byte per cell in LDS
constexpr int pstride(int side) { return r16((side * side + 1) / 2); }         // HBM ground bytes per env
constexpr int gstride(int side) { return 2 * pstride(side); }                  // byte-per-cell image bytes per env
// drl_step's LDS image of the ground: a byte per cell below DRL_GL_NIB_MIN_SIDE, the packed nibbles (the HBM
// row as is: half the LDS, so more waves fit a CU) from there on (round 6: C5's 64 x 64 envs, then C4's
// 32 x 32: 41.2 -> 39.7 us; at C3's 16 x 16 it measured slower, 29.3 -> 31.5 us, tools/ab.py)
#ifndef DRL_GL_NIB_MIN_SIDE
#define DRL_GL_NIB_MIN_SIDE 32
#endif
constexpr bool gl_nib(int side) { return side >= DRL_GL_NIB_MIN_SIDE; }
constexpr int glstride(int side) { return gl_nib(side) ? pstride(side) : gstride(side); }  // LDS ground bytes per env
constexpr int bm_bytes(int cells) { return r16((cells + 31) / 32 * 4); }       // occupancy bitmap
constexpr int paint_bytes(int k, int w) { return k > 0 ? r16(k * w * w) : 0; }  // observation paint
constexpr int nchg(int n_drones) { return 6 * n_drones + 2; }                  // changed-cell capacity
constexpr int chg_bytes(int n_drones) { return r16(2 * nchg(n_drones)); }
constexpr int bit_length(int v) { return v ? 1 + bit_length(v >> 1) : 0; }
#ifndef DRL_QN_RING
#define DRL_QN_RING 2
#endif
#ifndef DRL_QN_WAVES
#define DRL_QN_WAVES 8
#endif
// policy code of a W x W window (write_code_wave, the DRL_QNET code input):
// 4 groups of code_cpg cells, each padded to code_cpg8 u16 (16-B vectors)
constexpr int code_cpg(int W) { return (W * W + 3) / 4; }
constexpr int code_cpg8(int W) { return (code_cpg(W) + 7) / 8 * 8; }
constexpr int code_bytes(int W) { return 4 * code_cpg8(W) * 2; }
// layer 0's K-slices of a code-input net: 6 channels x code_cpg slots per lane group, 8 per slice, padded to the
// act kernels' slice ring
// layer 0's K order of a policy-code net, per lane group (drl_qnet_pack and every code act): slot sl <
// 6 * cpg holds observation channel code_slot_ch of the group's cell code_slot_cell.  The cell pairs (2p, 2p + 1),
// one dword of the code row each, take 12 consecutive slots, channel-major (slots 12p + 2ch, 12p + 2ch + 1), so
// one dword of the MFMA B operand is one channel of one code dword (drl_qnet_act_code4_kernel builds it with
// packed 16-bit operations); an odd count's last cell takes the 6 slots after the pairs; slot 6 * cpg carries
// the bias (lane group 0) and the slots after it are zero.
constexpr int code_slot_cell(int cpg, int sl) { return sl < 6 * (cpg & ~1) ? 2 * (sl / 12) + (sl & 1) : cpg - 1; }
constexpr int code_slot_ch(int cpg, int sl) { return sl < 6 * (cpg & ~1) ? (sl % 12) / 2 : sl - 6 * (cpg - 1); }
constexpr int code_kt(int W) { return ((6 * code_cpg(W) + 7) / 8 + DRL_QN_RING - 1) / DRL_QN_RING * DRL_QN_RING; }
constexpr int qn_ring = DRL_QN_RING;    // act kernel: K-slices in flight per wave (layer-0 slices padded to a multiple)
constexpr int qn_waves = DRL_QN_WAVES;  // act kernel: waves per workgroup (one workgroup per CU)
#ifndef DRL_QN_TILES
#define DRL_QN_TILES 2
#endif
constexpr int qn_tiles = DRL_QN_TILES;  // act kernel: 16-env tiles per pass sharing each weight fragment
// reset (wave kernel): the batched shuffle's bitmap of j's -- one bit per cell over a power-of-two
// count of words, at least 64 so that a chunk's ~46 ORs rarely share a word -- and its 64 i-slot words
constexpr int fy_bitmap_words(int cells) {
    int w = 64;
    while (w * 32 < cells) w *= 2;
    return w;
}
}  // namespace lay

enum : int { OBJ_EMPTY = 0, OBJ_SKYSCRAPER = 2, OBJ_STATION = 3, OBJ_DROPZONE = 4, OBJ_PACKET = 5 };

// n / d == umulhi(n, ceil(2^32 / d)) exactly for n * d < 2^32 (all our uses).
struct FastDiv {
    uint32_t m;
    int one;
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.one = (d == 1);
    f.m = f.one ? 0u : (uint32_t)((((uint64_t)1 << 32) + d - 1) / d);
    return f;
}

struct ObsGeom {
    int side, radius;
    uint32_t W, per, env_floats, gstride;
    FastDiv div_env, div_per, div_6, div_w, div_side;
};

struct StepArgs {
    int side, n_drones, gstride, kbits;  // gstride: LDS ground bytes per env (lay::glstride)
    int pstride, gl_nib;                 // packed HBM ground bytes per env; 1: the LDS image is packed nibbles
    int charge, discharge;
    float r_pickup, r_delivery, r_crash, r_charge;
    int64_t E;
    uint8_t* ground;
    uint32_t* drones;
    uint32_t* mt;
    uint32_t* mt_index;
    const int32_t* actions;
    float* rewards;
    uint8_t* dones;
    float* obs;
    int32_t* err;
    int wave_lds;   // LDS bytes per wave (= per block: one wave per block)
    int np;         // posidx entries per env (n_drones rounded up to 8)
    int lds_bm;     // bytes per env of the occupancy bitmap (16-B multiple)
    int lds_paint;  // bytes per env of the observation paint buffer (16-B multiple)
    int lds_chg;    // bytes per env of the changed-cell list (16-B multiple)
    int nchg;       // changed-cell list capacity (entries)
    int obs_k;      // observed drones (0: no observation)
    int obs_wide;   // observation stores: 1 = 16-B via LDS transpose, 0 = 3 x 8-B per cell
    int obs_nt;     // drl_step: 1 = streaming (non-temporal) observation stores (DRL_STEP_OBS_STREAM)
    int specialize; // 1: use a compile-time-geometry instance when one matches (DRL_SPECIALIZE=0 disables)
    int dones_packed; // 1: dones written as dwords (n_drones % 4 == 0, 4-B aligned rows and step strides)
    uint4* code;      // nullable: drone 0's policy code (lay::code_bytes(W) per env), written with the observation
    int code_lds;     // byte offset of the wave's code-row staging in its LDS (code non-NULL)
    // drl_step_code_replay: the step's drone-0 transitions land in a replay ring (a fused drl_replay_add; code
    // rows): env e (e >= ring_first) -> slot ring_base + e - ring_first (mod ring_cap); ring_next NULL: no ring
    uint4* ring_obs;
    uint4* ring_next;
    int32_t* ring_act;
    float* ring_rew;
    uint8_t* ring_done;
    const uint4* code_prev;  // the transitions' obs: the code rows the act read (not `code`)
    int64_t ring_first, ring_base, ring_cap;
    // drl_step_code_replay_synth (with the ring): drone indices >= 1 act as drl_synth_actions(synth_seed,
    // synth_step, env_offset) writes them, computed in the step; actions is read at column 0 only
    int synth;
    int64_t env_offset;
    uint64_t synth_seed, synth_step;
    uint32_t max_rounds;
    FastDiv div_side;
    ObsGeom og;
    // drl_rollout (several steps per launch, state resident on chip): steps and
    // per-step element strides of actions / rewards+dones / obs (0 = reuse)
    int steps;
    int64_t act_tstride, out_tstride, obs_tstride;
};

struct RefillArgs {
    int side, kbits;
    int list;  // 1: drl_refill_list_kernel (a per-workgroup worklist of the envs to convert); 0: one wave per env
    int64_t E;
    uint32_t* mt;
    uint32_t* mt_index;
};

struct ResetArgs {
    int side, n_drones, cells, gstride;  // gstride: packed HBM ground bytes per env (lay::pstride)
    int n_sky, n_pack, n_drop, n_stat;
    int64_t E;
    uint8_t* ground;
    uint32_t* drones;
    uint32_t* mt;
    uint32_t* mt_index;
    int reseed;
    uint64_t seed_base;
    const uint8_t* mask;
    int lanes, lane_lds, list_cap, block_lds, pool_branch;
    int wave_per_env, wave_lds;  // drl_reset_wave_kernel (large grids) and its LDS bytes
    int wpb;                     // ... envs (waves) per workgroup: 0 = the default, or 1, 2, 4, 8 (DRL_RESET_WPB)
    int fy_batch_min;            // wave kernel: shuffle 64 draws at a time while si >= this
    int fy_serial;               // ... i-range writers per chunk resolved by readlanes (more: table + jumps)
    int fy_bwords;               // ... words of its j bitmap (lay::fy_bitmap_words)
    FastDiv div_side;
};

// Q-network (dronerl_qnet.hip).  Layer 0 = input -> hidden[0], ..., layer
// n_hidden = last hidden -> actions.  Fragment offsets in 16-B units (one
// fragment = 64 lanes x 16 B), bias offsets in floats after the fragments.
constexpr int QN_MAX_LAYERS = 4;
struct QnetLayout {
    int n_layers;
    int nt[QN_MAX_LAYERS];        // 16-row output tiles
    int kt[QN_MAX_LAYERS];        // 32-wide K slices
    int in[QN_MAX_LAYERS], out[QN_MAX_LAYERS];
    int frag_off[QN_MAX_LAYERS];  // uint4 offset of the layer's fragments
    int bias_off[QN_MAX_LAYERS];  // float offset of the layer's biases (padded to 16 * nt)
    int frag_total;               // uint4s of fragments
    int n_bias;                   // floats of biases
    int lds_vec;                  // uint4s of the LDS image (fragments + biases)
    int precision;                // DRL_QNET_BF16 / DRL_QNET_F32
    int frag_lo_off[QN_MAX_LAYERS];  // F32: uint4 offset of the layer's lo fragments
    int total_vec;                // uint4s of the whole packed net
    int frag_src[QN_MAX_LAYERS];  // the pack kernel's contiguous element numbering of the hi fragments
    int bias_vec;                 // uint4 offset of the biases
    int lo0_lds;                  // F32: layer 0's hi and lo fragments are the LDS image (the rest is global)
    int code_w;                   // > 0: DRL_QNET_INPUT_CODE net of a code_w x code_w window
    int status_vec;               // uint4 offset of the pack status vector (the last one)
};

struct QnetPack {
    int n_layers;
    int frag_off[QN_MAX_LAYERS], kt[QN_MAX_LAYERS], in[QN_MAX_LAYERS], out[QN_MAX_LAYERS];
    int bias_off[QN_MAX_LAYERS];
    const float* w[QN_MAX_LAYERS];
    const float* b[QN_MAX_LAYERS];
    int64_t n_wfrag_elems, n_bias;
    uint16_t* packed_w;  // bf16 bits (F32: fp16 hi bits)
    float* packed_b;
    int precision;
    int frag_lo_off[QN_MAX_LAYERS];  // F32: lo fragments, uint4 offsets from packed_w
    int frag_src[QN_MAX_LAYERS];     // contiguous numbering of the hi elements (uint4 units) -> frag_off
    int code_w;                      // > 0: layer 0 in the policy code's K order for a code_w x code_w window
    int32_t* status;                 // the packed net's status word (DRL_ERR_QNET_RANGE: a weight outside fp16's range)
};

struct QnetArgs {
    int in_features, kt0, n_hidden, n_actions, precision;
    const float* eps_ptr;           // non-NULL: epsilon read from device memory (drl_qnet_act_eps; a learner's counter)
    int nt[QN_MAX_LAYERS];
    int frag_off[QN_MAX_LAYERS], bias_off[QN_MAX_LAYERS];
    int frag_total, lds_vec, n_bias;
    int frag_lo_off[QN_MAX_LAYERS];  // F32: lo fragments (uint4 offsets from packed, or in LDS: lo0_lds)
    int bias_vec, lo0_lds;           // biases' uint4 offset; F32 layout with layer 0 alone in LDS
    const uint4* packed;
    const float* obs;
    int64_t obs_stride, E;
    float epsilon;
    uint64_t seed, step;
    int64_t env_offset;
    int32_t* actions;
    int64_t action_stride;
    float* q;
    int synth_n;                    // > 1: also write drl_synth_actions' columns 1..synth_n-1
    uint64_t synth_seed, synth_step;
    int32_t* err;                   // F32: DRL_ERR_QNET_RANGE when an operand leaves fp16's range (nullable)
    int total_bytes;                // bytes of the packed net (code act: buffer loads of the later layers)
    int status_vec;                 // uint4 offset of the pack status vector (drl_qnet_pack's range flag)
};

struct ReplayArgs {
    int64_t first, n, cursor, capacity;
    int64_t base;  // slot of the first landing row: (cursor + first) % capacity
    int obs_floats;
    const float* obs;
    int64_t obs_stride;
    const float* next_obs;
    int64_t next_obs_stride;
    const int32_t* actions;
    int64_t action_stride;
    const float* rewards;
    int64_t reward_stride;
    const uint8_t* dones;
    int64_t done_stride;
    float* buf_obs;
    float* buf_next_obs;
    int32_t* buf_actions;
    float* buf_rewards;
    uint8_t* buf_dones;
};

// K index within a 32-wide slice of MFMA fragment element j for lane group g
// (dronerl_qnet.hip's header comment).
__host__ __device__ constexpr int qn_frag_k(int g, int j) { return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4); }

// Element e of layer l's hi fragments in drl_qnet_pack's numbering (fragment
// m * kt + t, lane, j) -> the weight W_l[row][k] it holds.  k == -1: layer 0's
// bias (the first padding slot of a code net's lane group 0); k outside
// [0, in) or row >= out: a zero pad.  Every real weight has exactly one slot.
struct PackSlot {
    int row, k;
};
__host__ __device__ inline PackSlot qnet_pack_slot(int l, int64_t e, int kt, int code_w, int in) {
    const int j = (int)(e & 7), lane = (int)((e >> 3) & 63);
    const int64_t frag = e >> 9;
    const int m = (int)(frag / kt), t = (int)(frag % kt);
    const int c = lane & 15, g = lane >> 4;
    PackSlot s{16 * m + c, 32 * t + qn_frag_k(g, j)};
    if (l == 0 && code_w > 0) {  // the policy code's K order (lay::code_slot_*)
        const int cpg = lay::code_cpg(code_w), cells = code_w * code_w, sl = 8 * t + j;
        const int lc = lay::code_slot_cell(cpg, sl), ch = lay::code_slot_ch(cpg, sl);
        const bool ok = sl < 6 * cpg && lc < cpg && g * cpg + lc < cells;
        s.k = ok ? (g * cpg + lc) * 6 + ch : in;
        if (g == 0 && sl == 6 * cpg) s.k = -1;
    }
    return s;
}

// The inverse: W_l[row][k] (k == -1: a code net's layer-0 bias) -> its
// element in layer l's fragments.
__host__ __device__ inline int64_t qnet_pack_elem(int l, int row, int k, int kt, int code_w) {
    int t, j, g;
    if (l == 0 && code_w > 0) {
        const int cpg = lay::code_cpg(code_w);
        int sl;
        if (k < 0) {  // the bias: lane group 0's first padding slot
            g = 0;
            sl = 6 * cpg;
        } else {
            const int cell = k / 6, ch = k - 6 * cell;
            g = (cell >= cpg) + (cell >= 2 * cpg) + (cell >= 3 * cpg);  // (cell < 4 cpg: no division)
            const int lc = cell - g * cpg;
            sl = lc < (cpg & ~1) ? 12 * (lc / 2) + 2 * ch + (lc & 1) : 6 * (cpg - 1) + ch;
        }
        t = sl / 8;
        j = sl % 8;
    } else {
        t = k / 32;
        const int kk = k % 32;
        g = kk < 16 ? kk / 4 : (kk - 16) / 4;
        j = kk < 16 ? kk % 4 : 4 + (kk - 16) % 4;
    }
    const int m = row / 16, c = row % 16;
    return (((int64_t)m * kt + t) * 64 + (g * 16 + c)) * 8 + j;
}

// Store weight w (W_l[row][k], or layer 0's bias for k == -1) at element e of
// layer l's fragments as drl_qnet_pack does: a code net's charge-channel
// weights carry the input's 1/100; DRL_QNET_F32 writes fp16 hi and lo =
// fp16((w - hi) * 2^11) (|w| >= 65504 or NaN raises DRL_ERR_QNET_RANGE in the
// packed net's status word), DRL_QNET_BF16 a bf16.
__device__ __forceinline__ void qnet_pack_store(const QnetPack& p, int l, int64_t e, float w) {
    if (p.precision == DRL_QNET_F32) {
        if (!(__builtin_fabsf(w) < 65504.0f)) atomicOr(p.status, DRL_ERR_QNET_RANGE);
        const _Float16 hi = (_Float16)w;
        reinterpret_cast<_Float16*>(p.packed_w)[(int64_t)p.frag_off[l] * 8 + e] = hi;
        reinterpret_cast<_Float16*>(p.packed_w)[(int64_t)p.frag_lo_off[l] * 8 + e] = (_Float16)((w - (float)hi) * 2048.0f);
    } else {
        reinterpret_cast<__bf16*>(p.packed_w)[(int64_t)p.frag_off[l] * 8 + e] = (__bf16)w;
    }
}
__device__ __forceinline__ void qnet_pack_write(const QnetPack& p, int l, int64_t e, int k, float w) {
    if (l == 0 && p.code_w > 0 && k >= 0 && k < p.in[l] && k % 6 == 4) w /= 100.0f;
    qnet_pack_store(p, l, e, w);
}
// The learner's table form (drl_dqn_init writes it): a weight's element in its layer's fragments in bits
// 0-30, bit 31 set where a code net's charge channel carries the input's 1/100.
__device__ __forceinline__ void qnet_pack_write_idx(const QnetPack& p, int l, uint32_t pe, float w) {
    if (pe >> 31) w /= 100.0f;
    qnet_pack_store(p, l, (int64_t)(pe & 0x7fffffffu), w);
}

// ----------------------------------------------------------- DQN learner ---
// (dronerl_learn.hip; include/dronerl.h drl_dqn_*.)  Device counters of the
// agent block: the layout include/dronerl.h documents as drl_dqn_counters.
struct DqnCounters {
    int32_t step, count;
    float epsilon, loss;
    double beta1_pow, beta2_pow;
    int32_t arrive, trained, target_due;
    float bc1, bc2;
    int32_t pad[3];
};
static_assert(sizeof(DqnCounters) == 64, "drl_dqn_counters is 64 bytes");

constexpr int DQN_MAX_BATCH = 64;
#ifndef DRL_DQN_TILE
#define DRL_DQN_TILE 4  // (8 until round 6: C3 train loop 69.3 -> 67.5 us per step with 4; 2: 68.6)
#endif
constexpr int DQN_TILE = DRL_DQN_TILE;  // layer-0 units per workgroup of the learner kernel
#ifndef DRL_DQN_THREADS
#define DRL_DQN_THREADS 1024  // (512 until round 6: C3 train loop 68.1 -> 66.6 us per step with 1024)
#endif
constexpr int DQN_THREADS = DRL_DQN_THREADS;  // the learner kernel's workgroup (DRL_DQN_THREADS: A/B knob)
constexpr int DQN_STAGE = 12;     // loads each thread keeps in flight when the learner stages data
constexpr int DQN_MAX_SEGS = 28;  // copy segments of the learner kernel's prefetch
constexpr int DQN_UB = 4;         // weights whose loads a thread issues together in the update phase
constexpr int DQN_PF = 8;         // weights per thread whose operands are loaded before the epoch wait
constexpr int DQN_W0R = 4096 / DQN_THREADS;  // layer-0 tile weights per thread in registers at the launch's start
                                             // (a tile of up to 8 units x up to 512 inputs)

// One segment of the learner kernel's one-round staging into LDS: element
// i < n lands at LDS float dst + (pad ? (i / row) * (row + pad) + i % row :
// i) (kind 4: in float4 units, dst still in floats).  kind 0: f32 (or raw
// 32-bit) at src[i]; 4: float4 at src[i]; the sampled rows' data through the
// per-row pointer table tbl (0 obs row, 1 next_obs row, 2 action, 3 reward,
// 4 done): kind 1: the 32-bit word at table[i]; 2: the u8 at table[i], as
// 0.0f / 1.0f; 3: element (b, k) = table[b][k], k < row; 5: float2 at
// src[i] (dst and pad in float2 units like kind 4's float4).  rm: the
// multiply-shift reciprocal of row (i / row == umulhi(i, rm); 0 when row == 1).
struct DqSeg {
    const void* src;
    int n, dst, row, pad, kind;
    uint32_t rm;
    int tbl;
};

struct LearnArgs {
    int n_layers, batch, code_w, trained, nblk0, tiles0, maxw;
    int in[QN_MAX_LAYERS], out[QN_MAX_LAYERS];
    int in4;                          // layer 0's input row stride in LDS / scratch (in[0] rounded up to 4)
    int xs0;                          // layer 0's weight row stride in LDS (>= in[0], = 4 mod 32: dq_mm1's banks)
    uint32_t rm_in, rm_rw;            // DqSeg::rm of in[0] and of row_words
    int ws_floats;                    // per-layer weight staging (no prefetch): max over l >= 1 of out_l * (in_l + 4)
    int region_a;                     // the tail workgroup's LDS floats before its prefetched tail (activations, masks)
    // prefetch != 0: every workgroup loads the last workgroup's data (later layers' weights of both nets,
    // every bias, the online biases' moments, the sampled rows' action / reward / done) into LDS after
    // region A in its first load round (tail[]); otherwise the last workgroup stages layer by layer
    int prefetch, ntail;
    int ntail_of[2];                  // the online tail's segments, then the target tail's (tail[ntail_of[0]..])
    int ntail_a, ntail_b;             // the online tail's: A before the forward pass, B behind it, C the rest
    DqSeg tail[DQN_MAX_SEGS];
    int tail_start[DQN_MAX_SEGS + 1];
    uint64_t* gmx;                    // scratch: max_a Q_target granules [batch] (the target tail's hand-off)
    int tw[2][QN_MAX_LAYERS], tb[2][QN_MAX_LAYERS], tm[QN_MAX_LAYERS], tv[QN_MAX_LAYERS], tr;  // LDS float offsets
    int twt[QN_MAX_LAYERS];           // (prefetch) W_l^T [in_l][out_l + 2], built by the online tail for the backward
    int64_t woff[QN_MAX_LAYERS], boff[QN_MAX_LAYERS];  // float offsets of W_l / b_l in a parameter set
    int64_t n_params;                 // floats of a parameter set
    float* online;
    float* target;
    float* adam_m;
    float* adam_v;
    DqnCounters* ctr;
    uint64_t* gz0;                    // scratch: layer-0 pre-activation granules [2 nets][batch][out0]
    uint64_t* gd1;                    // scratch: layer-1 delta granules [batch][out1] (the online layer-0 side)
    const uint32_t* pidx;             // scratch: each weight's packed-image element (qnet_pack_write_idx) [n_params]
    float* sh[QN_MAX_LAYERS];         // scratch: online hidden activations h_l [batch][out_l]
    float* sd[QN_MAX_LAYERS];         // scratch: deltas dL/dz_l [batch][out_l]
    // replay rows (buffers.py:79-93 sample)
    const uint32_t* r_obs;
    const uint32_t* r_next;
    int64_t row_words;
    const int32_t* r_act;
    const float* r_rew;
    const uint8_t* r_done;
    int64_t size, capacity;
    // fresh != 0: an add_many landing this step (rows f_first + off at slots f_base + off, off < f_rows) may
    // still be running: its rows are read from its own buffers (drl_replay_batch; strides in elements)
    int fresh;
    int64_t f_base, f_rows, f_first;
    const uint32_t* f_obs;
    const uint32_t* f_next;
    const int32_t* f_act;
    const float* f_rew;
    const uint8_t* f_done;
    int64_t f_obs_stride, f_next_stride, f_act_stride, f_rew_stride, f_done_stride;
    uint64_t seed;
    // hyperparameters, as the f32 constants jax's weak typing makes of the python floats
    float gamma, b1, b2, c1, c2, adam_eps, neg_lr, tau, one_minus_tau, eps_decay, eps_end, inv_batch;
    double b1d, b2d;
    int target_every, eps_every;
    // the act kernels' packed image of the online net (the learner refreshes it)
    QnetPack pack;
    int64_t wstart[QN_MAX_LAYERS + 1];  // the weights in set order: index of layer l's first; [L] = their total
    uint64_t* stamps;                   // DRL_DQN_STAMPS builds: [8 per workgroup (<= 64)][512 + last workgroup's]
    // bounded waits: polls of a hand-off word / of a granule before a workgroup gives up (DqnCounters::pad[0])
    uint32_t spin_word, spin_granule;
    int drop_handoff;                   // debug knob (DRL_DQN_DEBUG_DROP_HANDOFF): the online tail omits the epoch word
};
constexpr uint32_t DQN_SPIN_WORD = 1u << 24, DQN_SPIN_GRANULE = 1u << 22;

// co-residency of the learner's workgroups (they poll each other's hand-offs): how many can be resident at
// once on this device with `lds` bytes of dynamic LDS each (occupancy x compute units)
int dqn_train_resident_capacity(size_t lds, int num_cus);

hipError_t launch_qnet_pack(const QnetPack& p, hipStream_t s);
hipError_t launch_dqn_train(const LearnArgs& a, size_t lds_grad, hipStream_t s);
hipError_t launch_dqn_init(void* counters, float epsilon, hipStream_t s);
hipError_t launch_dqn_sample(const void* counters, uint64_t seed, int batch, int64_t size, int64_t* out, hipStream_t s);
hipError_t launch_qnet_act(const QnetArgs& a, int num_cus, hipStream_t s);
hipError_t launch_qnet_act_code(const QnetArgs& a, int window, int num_cus, hipStream_t s);
hipError_t launch_replay_add(const ReplayArgs& a, hipStream_t s);

enum StepMode : int { kStepMode = 0, kObsMode = 1, kRolloutMode = 2 };
hipError_t launch_step(const StepArgs& a, int P, hipStream_t s, int mode);
hipError_t launch_reset(const ResetArgs& a, hipStream_t s);
hipError_t launch_decode(const uint32_t* drones, int64_t E, int N, int32_t* order, int32_t* y, int32_t* x,
                         int32_t* c, uint8_t* k, hipStream_t s);
hipError_t launch_code_decode(const void* code, int64_t n, int W, float* obs, hipStream_t s);
hipError_t launch_hbm_probe(const void* src, void* dst, int64_t bytes, int mode, int num_cus, hipStream_t s);
hipError_t launch_ground_unpack(const uint8_t* packed, int pstride, uint8_t* out, int cells, int64_t E, hipStream_t s);
hipError_t launch_ground_pack(const uint8_t* in, int cells, uint8_t* packed, int pstride, int64_t E, int32_t* err,
                              hipStream_t s);
hipError_t launch_grid_obs(const uint8_t* ground, const uint32_t* drones, int64_t E, int side, int N, int gstride,
                           float* out, hipStream_t s);
hipError_t launch_encode(uint32_t* drones, int64_t E, int N, const int32_t* order, const int32_t* y,
                         const int32_t* x, const int32_t* c, const uint8_t* k, hipStream_t s);
hipError_t launch_refill(const RefillArgs& a, hipStream_t s);
hipError_t launch_mt_get(const uint32_t* mt, const uint32_t* mt_index, int64_t E, uint32_t* out, hipStream_t s);
hipError_t launch_mt_set(uint32_t* mt, uint32_t* mt_index, int64_t E, const uint32_t* in, int32_t* err, hipStream_t s);
hipError_t launch_synth(uint64_t seed, uint64_t step, int64_t env_offset, int64_t E, int N, int32_t* out,
                        hipStream_t s);

}  // namespace drl
