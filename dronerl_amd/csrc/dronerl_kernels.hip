// dronerl_kernels.hip — batched DroneRL env kernels for MI355X (gfx950, CDNA4).
//
// Semantics: nyx-ai/droneRL torch_impl (env.py:68-233, wrappers.py:10-73),
// bit-exact including each env's CPython MT19937 draw stream.  Layout and
// design: DESIGN.md.  Summary:
//
//  drl_step_kernel<P>  one wavefront lane per (env, drone slot); an env owns a
//      group of P lanes (P = pow2 >= n_drones), 64/P envs per wave, one wave
//      per block.  Slots are kept in dict order O, so "earlier in O" is "lower
//      lane".  The env's ground is staged into LDS by LDS-DMA, first-comer
//      claims / crash ordering are resolved with DPP lane swaps (8/16-lane
//      groups) or __shfl, and __ballot, and the serial respawn section
//      (env.py:186-210) draws D*P MT outputs per round in parallel and places
//      items from the accepted (y, x) pairs with ballots.  The observation
//      window is written from LDS with 16-B stores (streaming on request).
//  drl_rollout_kernel<P>  the same per step, several steps per launch with
//      the state on chip (P >= 16; narrower groups roll out as drl_step
//      launches).
//  drl_obs_kernel<P>   the same geometry, observation only.
//  drl_reset_wave_kernel  one wavefront per env: MT state in registers,
//      batched Fisher-Yates shuffles (64 draws per step) over an LDS list.
//  drl_reset_kernel    one lane per env (the A/B alternative): the shuffle
//      list lives in LDS, MT twists are done cooperatively by the whole wave.
//  drl_refill_list_kernel  the respawn-candidate rings: per 32 envs, the ones
//      whose stream reached the ring's last block get a wave that converts
//      the next MT block in registers (drl_refill_kernel: one wave per env).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronerl_internal.h"

namespace drl {

// Diagnostic build only (-DDRL_STAMPS, tools/stamps.py): per-wave phase
// timestamps (s_memtime) into a debug buffer.  Never compiled into the product.
#ifdef DRL_STAMPS
__device__ unsigned long long* g_stamps;
#define DRL_STAMP(i)                                                                     \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        unsigned long long t_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
        const int64_t sw_ = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); \
        if ((threadIdx.x & 63) == 0 && g_stamps) g_stamps[sw_ * 16 + (i)] = t_;          \
        if ((threadIdx.x & 63) == 0 && g_stamps && ((i) == 0 || (i) == 6))               \
            g_stamps[sw_ * 16 + 8 + (i) / 6] = __builtin_amdgcn_s_memrealtime();         \
        __builtin_amdgcn_sched_barrier(0);                                               \
    } while (0)
// sub-phase clock (accumulated per wave into slots 10..13 of the stamp row)
#define DRL_SUBT(v)                                                                  \
    do {                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");   \
        __builtin_amdgcn_sched_barrier(0);                                           \
    } while (0)
// reset: clocks accumulated per category (uniform, in SGPRs), written at the end
#define DRL_RS_DECL unsigned long long rs_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, rs_t0 = 0, rs_t1 = 0, rs_tt = 0
#define DRL_RS_BEGIN() DRL_SUBT(rs_t0)
#define DRL_RS_END(k)           \
    do {                        \
        DRL_SUBT(rs_t1);        \
        rs_acc[k] += rs_t1 - rs_t0; \
    } while (0)
#define DRL_RS_COUNT(k) (++rs_acc[k])
#else
#define DRL_STAMP(i) \
    do {             \
    } while (0)
#define DRL_SUBT(v) \
    do {            \
    } while (0)
#define DRL_RS_DECL
#define DRL_RS_BEGIN() \
    do {               \
    } while (0)
#define DRL_RS_END(k) \
    do {              \
    } while (0)
#define DRL_RS_COUNT(k) \
    do {                \
    } while (0)
#endif

// LDS pointer types: address arithmetic on them stays 32-bit (generic
// pointers into LDS cost 64-bit math and registers the 64-VGPR kernels lack)
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(3))) uint16_t l_u16;
typedef __attribute__((address_space(3))) uint32_t l_u32;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 l_u2;
typedef __attribute__((address_space(3))) u32x4 l_u4;
typedef __attribute__((address_space(3))) f32x2 l_f2;

// ---------------------------------------------------------------- helpers ---
__device__ __forceinline__ void wave_sync() {
    // LDS traffic inside one wavefront is processed in order; this keeps the
    // compiler from moving LDS accesses across the point.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// L1-bypassing (sc1, L2-served) load: MT words may have been rewritten by a
// twist earlier in the same launch.
__device__ __forceinline__ uint32_t load_l2(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int bitlen(uint32_t n) { return 32 - __clz((int)n); }

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv d) {
    return d.one ? n : __umulhi(n, d.m);
}

__device__ __forceinline__ uint32_t pack_drone(int y, int x, int c, int carry, int idx) {
    return (uint32_t)y | ((uint32_t)x << 8) | ((uint32_t)c << 16) | ((uint32_t)carry << 24) |
           ((uint32_t)idx << 25);
}

// MT19937 twist of one env's state held by all 64 lanes of the wave in
// registers: lane l holds x[c] = mt[64c + l].  Chunks are processed in
// ascending order, each computed from old/new values exactly as the sequential
// generator sees them: mt[i+1] and mt[i+397] (i < 227) are still old (chunks
// > c), mt[i-227] (i >= 227) and mt[0] (i = 623) are already new (chunks < c).
// Lane offsets are constants (397 = 6*64 + 13, 227 = 4*64 - 29).
__device__ __forceinline__ void twist_regs(uint32_t (&x)[10], int lane) {
    // mt[i+397] (old) or mt[i-227] (new): one bpermute per chunk, the source
    // register chosen by the SENDING lane (the two source chunks occupy
    // disjoint lane ranges); chunk 3 straddles i = 227 and takes two.  The
    // bpermutes go out in four batches, each as soon as its sources are final
    // (chunks 0-2 and 3's old half read old chunks 6-9; 3's new half, 4 and 5
    // read new 0-2; 6-8 read new 2-5; 9 reads new 5-6).
    // (the empty asm pins both sources in registers: folded into a select of
    // addresses, the array would be indexed per lane and live in scratch)
    auto pick = [&](bool lo, uint32_t a, uint32_t b) __attribute__((always_inline)) {
        asm("" : "+v"(a), "+v"(b));
        return lo ? a : b;
    };
    auto far_old = [&](int c) __attribute__((always_inline)) {
        return (uint32_t)__shfl(pick(lane < 13, x[c + 7], x[c + 6]), (lane + 13) & 63);
    };
    auto far_new = [&](int c) __attribute__((always_inline)) {
        return (uint32_t)__shfl(pick(lane < 29, x[c - 3], x[c - 4]), (lane + 29) & 63);
    };
    auto step = [&](int c, uint32_t far) __attribute__((always_inline)) {
        // mt[i+1]: DPP wave_shl:1 (lane l reads lane l+1); lane 63 takes lane 0
        // of the next (old) chunk, and word 623 the new mt[0]
        uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[c], 0x130, 0xf, 0xf, false);
        if (c < 9) {
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)x[c + 1], 0);
            if (lane == 63) nxt = n0;
        } else {
            const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)x[0], 0);
            if (lane == MT_N - 1 - 576) nxt = m0;
        }
        const uint32_t y = (x[c] & 0x80000000u) | (nxt & 0x7fffffffu);
        x[c] = far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    };
    const uint32_t f0 = far_old(0), f1 = far_old(1), f2 = far_old(2);
    const uint32_t f3o = (uint32_t)__shfl(x[9], (lane + 13) & 63);
    step(0, f0);
    step(1, f1);
    step(2, f2);
    const uint32_t f3n = (uint32_t)__shfl(x[0], (lane + 29) & 63);
    const uint32_t f4 = far_new(4), f5 = far_new(5);
    step(3, lane < MT_N - MT_M - 192 ? f3o : f3n);
    step(4, f4);
    step(5, f5);
    const uint32_t f6 = far_new(6), f7 = far_new(7), f8 = far_new(8);
    step(6, f6);
    step(7, f7);
    step(8, f8);
    step(9, far_new(9));
}

// In-place twist of the env row in global memory (register-resident).
__device__ __noinline__ void twist_wave(uint32_t* row, int lane) {
    uint32_t x[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int i = 64 * c + lane;
        x[c] = (i < MT_N) ? load_l2(row + i) : 0u;
    }
    twist_regs(x, lane);
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int i = 64 * c + lane;
        if (i < MT_N) row[i] = x[c];
    }
    // make the rewritten words visible to this workgroup's later sc1 loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
}

// n / D for n <= NMAX (compile-time) as one multiply and a shift: the
// smallest shift whose rounded-up reciprocal is exact over [0, NMAX].
struct SmallDiv {
    uint32_t m;
    int s;
};
constexpr SmallDiv find_small_div(uint32_t d, uint32_t nmax) {
    for (int s = 0; s < 32; ++s) {
        const uint64_t m = ((1ull << s) + d - 1) / d;
        if (m * nmax >= (1ull << 24)) break;  // keep v_mul_u32_u24
        bool ok = true;
        for (uint32_t n = 0; n <= nmax && ok; ++n) ok = ((n * m) >> s) == n / d;
        if (ok) return SmallDiv{(uint32_t)m, s};
    }
    return SmallDiv{0, -1};  // none: callers fall back to n / d
}
template <uint32_t D, uint32_t NMAX>
__device__ __forceinline__ uint32_t small_div(uint32_t n) {
    constexpr SmallDiv sd = find_small_div(D, NMAX);
    if constexpr (sd.s < 0) return n / D;
    else if constexpr (sd.m == 1) return n >> sd.s;
    else return __umul24(n, sd.m) >> sd.s;
}

// c / 100.0f, correctly rounded, for integer c in [0, 255]: one multiply and
// two FMA corrections (checked exhaustively against the IEEE quotient with
// exact rational arithmetic), instead of the full f32 division sequence.
__device__ __forceinline__ float div100(int c) {
    const float x = (float)c;
    const float r = 0.01f;
    const float q = x * r;
    const float e = __fmaf_rn(-q, 100.0f, x);
    return __fmaf_rn(e, r, q);
}

// ------------------------------------------------------------- geometry ---
// Geometry of a step/obs launch.  The benchmark shapes get instances with the
// side (GC), drone count (NC), window radius (RC) and observed-drone count (KC,
// 0 = no observation) as compile-time constants, so LDS offsets, divisions by
// side / window and loop bounds fold; every other shape runs the GC = NC = RC
// = 0, KC = -1 instance, which reads them from StepArgs.  Both derive the LDS
// layout from the same lay:: formulas as the host.
template <int GC, int NC, int RC, int KC>
struct Geo {
    const StepArgs& a;
    __device__ int side() const { return GC > 0 ? GC : a.side; }
    __device__ uint32_t div_side(uint32_t n) const { return GC > 0 ? n / (uint32_t)GC : fdiv(n, a.div_side); }
    __device__ int kbits() const { return GC > 0 ? lay::bit_length(GC) : a.kbits; }
    __device__ int gstride() const { return GC > 0 ? lay::glstride(GC) : a.gstride; }      // LDS ground bytes / env
    __device__ int pstride() const { return GC > 0 ? lay::pstride(GC) : a.pstride; }       // HBM ground bytes / env
    __device__ bool nib() const { return GC > 0 ? lay::gl_nib(GC) : a.gl_nib != 0; }       // packed LDS image
    __device__ int lds_bm() const { return GC > 0 ? lay::bm_bytes(GC * GC) : a.lds_bm; }
    __device__ int n() const { return NC > 0 ? NC : a.n_drones; }
    __device__ int np() const { return NC > 0 ? lay::np(NC) : a.np; }
    __device__ int nchg() const { return NC > 0 ? lay::nchg(NC) : a.nchg; }
    __device__ int lds_chg() const { return NC > 0 ? lay::chg_bytes(NC) : a.lds_chg; }
    __device__ int K() const { return KC >= 0 ? KC : a.obs_k; }
    __device__ int radius() const { return RC > 0 ? RC : a.og.radius; }
    __device__ uint32_t W() const { return RC > 0 ? (uint32_t)(2 * RC + 1) : a.og.W; }
    __device__ int lds_paint() const { return (RC > 0 && KC >= 0) ? lay::paint_bytes(KC, 2 * RC + 1) : a.lds_paint; }
    // observation: window cells per env (K windows) and divisions by it / a window / its width
    // (arguments: q < 16 envs x env_cells; a cell index within K windows; within one window)
    static constexpr uint32_t kW = RC > 0 ? 2 * RC + 1 : 1, kCells = KC > 0 ? KC * kW * kW : 1;
    __device__ uint32_t env_cells() const { return (RC > 0 && KC > 0) ? kCells : a.og.env_floats / 6u; }
    __device__ uint32_t div_env(uint32_t n) const {
        if constexpr (RC > 0 && KC > 0) return small_div<kCells, 16 * kCells>(n);
        else return fdiv(n, a.og.div_env);
    }
    __device__ uint32_t div_win(uint32_t n) const {
        if constexpr (KC == 1) return 0u;
        else if constexpr (RC > 0 && KC > 0) return small_div<kW * kW, kCells>(n);
        else return fdiv(n, a.og.div_per);
    }
    __device__ uint32_t div_w(uint32_t n) const {
        if constexpr (RC > 0) return small_div<kW, kW * kW>(n);
        else return fdiv(n, a.og.div_w);
    }
    static constexpr bool kObs = KC != 0;  // KC == 0: instance for steps without observation
    static constexpr int kN = NC;
    static constexpr int kGstride = GC > 0 ? lay::glstride(GC) : 0;
    static constexpr int kPstride = GC > 0 ? lay::pstride(GC) : 0;
};
using GeoRT = Geo<0, 0, 0, -1>;

// ------------------------------------------------------------ LDS image ---
// Per-wave LDS image of its GPW envs; every region is [GPW][stride] with
// 16-byte strides (lay:: / Geo):
//   gl     u8  [gstride]  ground codes (staged by LDS-DMA, env-major = HBM order)
//   paint  u8  [K*W*W]    air byte (charge+1)|carry<<7 of drones inside each observed window
//   posidx u16 [np]       cell of drone index k
//   -- scratch, dead once the step is written back; the observation's
//      transpose stage (OBS_U*1536 B per wave) aliases it --
//   bm     u32 [bm]       drone-occupancy bitmap of the cells (respawn mask)
//   stash  u32 [P]        drl_rollout: the drone records between steps (O order)
//   chg    u16 [nchg]     ground cells changed this step (written back as bytes)
//   cnt    u32 [4]        chg count
struct WaveLds {
    l_u8* gl;
    l_u8* paint;
    l_u16* posidx;
    l_u32* bm;
    l_u32* stash;
    l_u16* chg;
    l_u32* cnt;
    l_u8* stage;
};

template <class GEO>
__device__ __forceinline__ WaveLds carve(l_u8* wb, int gpw, int P, const GEO& g) {
    WaveLds w;
    w.gl = wb;
    wb += gpw * g.gstride();
    w.paint = wb;
    wb += gpw * g.lds_paint();
    w.posidx = reinterpret_cast<l_u16*>(wb);
    wb += gpw * g.np() * 2;
    w.stage = wb;
    w.bm = reinterpret_cast<l_u32*>(wb);
    wb += gpw * g.lds_bm();
    w.stash = reinterpret_cast<l_u32*>(wb);
    wb += gpw * P * 4;
    w.chg = reinterpret_cast<l_u16*>(wb);
    wb += gpw * g.lds_chg();
    w.cnt = reinterpret_cast<l_u32*>(wb);
    return w;
}

// The ground is packed in HBM (one nibble per cell, ABI 8: half the bytes of
// the round-3 byte layout) and unpacked into a byte per cell in LDS: a packed
// 16-B vector holds 32 cells, which go to 32 LDS bytes (the LDS row is twice
// the packed row, so the wave's rows stay contiguous in both).
__device__ __forceinline__ void nib_unpack_store(l_u8* dst, const uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = w[k] & 0x0f0f0f0fu, hi = (w[k] >> 4) & 0x0f0f0f0fu;
        o[2 * k] = __builtin_amdgcn_perm(hi, lo, 0x05010400u);      // cells 8k+0..3
        o[2 * k + 1] = __builtin_amdgcn_perm(hi, lo, 0x07030602u);  // cells 8k+4..7
    }
    reinterpret_cast<l_u4*>(dst)[0] = u32x4{o[0], o[1], o[2], o[3]};
    reinterpret_cast<l_u4*>(dst)[1] = u32x4{o[4], o[5], o[6], o[7]};
}

// 32 LDS bytes (cells < 16) -> the packed 16-B vector
__device__ __forceinline__ uint4 nib_pack_load(const l_u8* src) {
    const u32x4 a = reinterpret_cast<const l_u4*>(src)[0], b = reinterpret_cast<const l_u4*>(src)[1];
    const uint32_t c[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t0 = c[2 * k] | (c[2 * k] >> 4), t1 = c[2 * k + 1] | (c[2 * k + 1] >> 4);
        o[k] = __builtin_amdgcn_perm(t1, t0, 0x06040200u);  // bytes 0 and 2 of each
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// The wave's packed grounds (contiguous in HBM, env-major, nbytes) -> LDS,
// runtime geometry: load, unpack, store.
__device__ __forceinline__ void stage_ground_nib(const uint8_t* __restrict__ src, int nbytes, l_u8* gl, int lane,
                                                 bool nib) {
    const int nvec = nbytes / 16;
    for (int v = lane; v < nvec; v += 64) {
        const uint4 x = reinterpret_cast<const uint4*>(src)[v];
        if (nib) reinterpret_cast<l_u4*>(gl)[v] = u32x4{x.x, x.y, x.z, x.w};  // (the packed row as is)
        else nib_unpack_store(gl + v * 32, x);
    }
}

// Compile-time form in two halves: the loads (NV vectors, unrolled, so the
// compiler counts them; vectors past the wave's valid envs re-read the last
// valid vector and unpack into LDS the wave does not use) are issued with the
// step's first loads, the unpack and LDS stores come after the claim scan,
// which does not need the ground, so the loads' latency overlaps it.
// NT: streaming (non-temporal) loads -- the large grids' rows (lay::gl_nib sides: C5's 2 KB per env), which
// would otherwise push the step's outputs the next kernels read out of the caches (C5 train loop, one box:
// step 113.2 -> 110.4 us, learner 28.7 -> 26.2; C3 slower, 16.6 -> 17.5: byte-image sides keep cached loads)
template <int NV, bool NT = false>
struct NibStage {
    static constexpr int Q = (NV + 63) / 64;
    uint4 v[Q];
    __device__ __forceinline__ void load(const uint8_t* __restrict__ src, int nbytes, int lane) {
        const uint32_t last = (uint32_t)(nbytes / 16 - 1);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if constexpr (NT) {
                const u32x4 t =
                    __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + min((uint32_t)(64 * q + lane), last));
                v[q] = make_uint4(t[0], t[1], t[2], t[3]);
            } else {
                v[q] = reinterpret_cast<const uint4*>(src)[min((uint32_t)(64 * q + lane), last)];
            }
        }
    }
    __device__ __forceinline__ void store(l_u8* gl, int lane, bool nib) const {
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (NV % 64 == 0 || 64 * q + lane < NV) {
                if (nib) reinterpret_cast<l_u4*>(gl)[64 * q + lane] = u32x4{v[q].x, v[q].y, v[q].z, v[q].w};
                else nib_unpack_store(gl + (64 * q + lane) * 32, v[q]);
            }
    }
};

// packed-ground nibble access in HBM (reset; grid observation)
__device__ __forceinline__ uint32_t nib_get(const uint8_t* row, int cell) {
    return (row[cell >> 1] >> ((cell & 1) * 4)) & 15u;
}
__device__ __forceinline__ void nib_or(uint8_t* row, int cell, uint32_t code) {  // the cell's nibble is 0
    atomicOr(reinterpret_cast<uint32_t*>(row) + (cell >> 3), code << ((cell & 7) * 4));
}
__device__ __forceinline__ uint32_t nib_get_l2(uint8_t* row, int cell) {  // after nib_or: read at L2
    const uint32_t w = __hip_atomic_load(reinterpret_cast<uint32_t*>(row) + (cell >> 3), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return (w >> ((cell & 7) * 4)) & 15u;
}
__device__ __forceinline__ void nib_clear(uint8_t* row, int cell) {
    atomicAnd(reinterpret_cast<uint32_t*>(row) + (cell >> 3), ~(15u << ((cell & 7) * 4)));
}

// One env's ground in drl_step's LDS image (GEO::nib(): packed nibbles, the HBM row as is, else a byte per
// cell).  Nibble writes are LDS atomics on the cell's dword (two lanes may change two cells of one dword).
template <class GEO>
__device__ __forceinline__ int gl_get(const GEO& g, const l_u8* gl, int cell) {
    if (g.nib()) return (gl[cell >> 1] >> ((cell & 1) << 2)) & 15;
    return gl[cell];
}
template <class GEO>
__device__ __forceinline__ void gl_clear(const GEO& g, l_u8* gl, int cell) {  // -> OBJ_EMPTY
    if (g.nib()) __atomic_fetch_and(reinterpret_cast<l_u32*>(gl) + (cell >> 3), ~(15u << ((cell & 7) << 2)),
                                    __ATOMIC_RELAXED);
    else gl[cell] = OBJ_EMPTY;
}
template <class GEO>
__device__ __forceinline__ void gl_put(const GEO& g, l_u8* gl, int cell, int obj) {  // an OBJ_EMPTY cell -> obj
    if (g.nib()) __atomic_fetch_or(reinterpret_cast<l_u32*>(gl) + (cell >> 3), (uint32_t)obj << ((cell & 7) << 2),
                                   __ATOMIC_RELAXED);
    else gl[cell] = (uint8_t)obj;
}

// 16-B observation store.  NT: streaming (global_store_dwordx4 ... nt), for
// drl_rollout, whose per-step observations are bulk output (C3 rollout 29.4
// -> 26.2 us/step).  drl_step keeps ordinary stores: its observation is read
// right away by the next kernel (the policy), which then hits the MALL (C3
// train loop 73.6 us/step cached vs 76.5 streaming, although the step alone
// is 11% faster streaming).
template <bool NT>
__device__ __forceinline__ void store_obs16(uint4* p, u32x4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<u32x4*>(p) = v;
    }
}

// Zero [nbytes) of LDS (16-B multiple) cooperatively.
template <class T>
__device__ __forceinline__ void lds_zero(T* p, int nbytes, int lane) {
    l_u4* q = reinterpret_cast<l_u4*>(p);
    for (int v = lane; v < nbytes / 16; v += 64) q[v] = (u32x4){0u, 0u, 0u, 0u};
}

// ------------------------------------------------------- observation write ---
// WindowedGridView windows (wrappers.py:10-31,55-73) of the wave's envs:
// lane = one window cell; its 6 channels are computed branch-free and stored
// as three 8-B pieces (consecutive lanes cover a contiguous span).  ch0 drone,
// ch1 packet OR carrying drone, ch2 dropzone, ch3 station, ch4 charge/100
// (true f32 division, == f32(double c/100)), ch5 skyscraper or wall.
// `base` is the wave's first observation float (16-B aligned unless a wave
// holds one env with an odd K*W*W).
// CODE: also store drone 0's policy code (include/dronerl.h drl_step_code;
// `code` = the wave's first env's code row): each lane of a k = 0 cell puts
// its u16 (object | air << 3) at its group slot of an LDS copy of the wave's
// code rows (`cst`, zeroed first: the padding), and the rows leave as 16-B
// stores after the last pass.  F32 = false: the code alone (no f32
// observation; `base` unused).
template <bool NT = false, bool CODE = false, bool F32 = true, class GEO>
__device__ __forceinline__ void write_obs_wave(float* __restrict__ base, int nenv_w, const GEO& g, const WaveLds& w,
                                               bool obs_wide, int lane, uint16_t* __restrict__ code = nullptr,
                                               l_u16* cst = nullptr) {
    static_assert(CODE || F32, "nothing to write");
    const uint32_t W = g.W();
    const uint32_t win = W * W;
    const uint32_t env_cells = g.env_cells();  // K * W*W
    const uint32_t ncell = (uint32_t)nenv_w * env_cells;
    const int G = g.side(), R = g.radius();
    const uint32_t gstride = (uint32_t)g.gstride(), np = (uint32_t)g.np(), lpaint = (uint32_t)g.lds_paint();
    const bool wide = obs_wide && ((uintptr_t)base & 15u) == 0;
    const int cpg = lay::code_cpg((int)W), cpg8 = lay::code_cpg8((int)W);
    if constexpr (CODE) {
        lds_zero(cst, nenv_w * 8 * cpg8, lane);
        wave_sync();
    }
    for (uint32_t q0 = 0; q0 < ncell; q0 += 64 * OBS_U) {
        uint32_t e[OBS_U], rem[OBS_U], wy[OBS_U], wx[OBS_U], pos[OBS_U];
#pragma unroll
        for (int u = 0; u < OBS_U; ++u) {
            const uint32_t q = min(q0 + (uint32_t)(lane + 64 * u), ncell - 1u);
            e[u] = g.div_env(q);
            rem[u] = q - e[u] * env_cells;
            const uint32_t k = g.div_win(rem[u]);
            const uint32_t c = rem[u] - k * win;
            wy[u] = g.div_w(c);
            wx[u] = c - wy[u] * W;
            pos[u] = w.posidx[e[u] * np + k];
        }
        float2 v[OBS_U][3];
#pragma unroll
        for (int u = 0; u < OBS_U; ++u) {
            const uint32_t py = g.div_side(pos[u]);
            const uint32_t px = pos[u] - py * (uint32_t)G;
            const int y = (int)(py + wy[u]) - R;
            const int x = (int)(px + wx[u]) - R;
            const bool in = (unsigned)y < (unsigned)G && (unsigned)x < (unsigned)G;
            const uint32_t o = (uint32_t)gl_get(g, w.gl + e[u] * gstride, in ? y * G + x : 0);
            const uint32_t obj = in ? o : (uint32_t)OBJ_SKYSCRAPER;
            const uint32_t air = w.paint[e[u] * lpaint + rem[u]];
            if constexpr (CODE) {
                if (rem[u] < win) {  // drone index 0's window (k = 0)
                    const uint32_t cl = rem[u], grpc = cl / (uint32_t)cpg;
                    cst[e[u] * (uint32_t)(4 * cpg8) + grpc * (uint32_t)(cpg8 - cpg) + cl] = (uint16_t)(obj | (air << 3));
                }
            }
            if constexpr (!F32) continue;
            v[u][0].x = air ? 1.0f : 0.0f;
            v[u][0].y = (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f;
            v[u][1].x = obj == OBJ_DROPZONE ? 1.0f : 0.0f;
            v[u][1].y = obj == OBJ_STATION ? 1.0f : 0.0f;
            v[u][2].x = air ? div100((int)(air & 0x7fu) - 1) : 0.0f;
            v[u][2].y = obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f;
        }
        if constexpr (!F32) continue;
        if (wide) {
            // transpose through LDS: lane u*64+l's 24 B at stage[(u*64+l)*24], then 16-B stores
            l_f2* st = reinterpret_cast<l_f2*>(w.stage);
#pragma unroll
            for (int u = 0; u < OBS_U; ++u) {
                const int slot = (u * 64 + lane) * 3;
                st[slot] = (f32x2){v[u][0].x, v[u][0].y};
                st[slot + 1] = (f32x2){v[u][1].x, v[u][1].y};
                st[slot + 2] = (f32x2){v[u][2].x, v[u][2].y};
            }
            wave_sync();
            const l_u4* sv = reinterpret_cast<const l_u4*>(w.stage);
            uint4* dst = reinterpret_cast<uint4*>(base + 6u * q0);
            if (q0 + 64u * OBS_U <= ncell) {  // full pass: 96*OBS_U 16-B pieces
#pragma unroll
                for (int t = 0; t < 96 * OBS_U; t += 64)
                    if (96 * OBS_U - t >= 64 || lane < 96 * OBS_U - t) store_obs16<NT>(&dst[t + lane], sv[t + lane]);
            } else {
                const uint32_t nbytes = (ncell - q0) * 24u;
                for (uint32_t t = lane; t * 16u < nbytes; t += 64) {
                    if (t * 16u + 16u <= nbytes) {
                        store_obs16<NT>(&dst[t], sv[t]);
                    } else {  // 8-byte tail
                        reinterpret_cast<u32x2*>(dst + t)[0] = reinterpret_cast<const l_u2*>(sv + t)[0];
                    }
                }
            }
            wave_sync();
        } else {
#pragma unroll
            for (int u = 0; u < OBS_U; ++u) {
                const uint32_t q = q0 + (uint32_t)(lane + 64 * u);
                if (q < ncell) {
                    float2* o = reinterpret_cast<float2*>(base + 6u * q);
                    o[0] = v[u][0];
                    o[1] = v[u][1];
                    o[2] = v[u][2];
                }
            }
        }
    }
    if constexpr (CODE) {  // the wave's code rows: nenv_w * cpg8 / 2 16-B vectors
        wave_sync();
        const l_u4* cv = reinterpret_cast<const l_u4*>(cst);
        uint4* dst = reinterpret_cast<uint4*>(code);
        for (int v = lane; v < nenv_w * cpg8 / 2; v += 64) {
            const u32x4 x = cv[v];
            dst[v] = make_uint4(x[0], x[1], x[2], x[3]);
        }
    }
}

// Policy code (include/dronerl.h drl_step_code): drone index 0's window as one
// u16 per cell -- object code (bits 0-2; walls read as skyscrapers) | air byte
// << 3 ((charge+1) | carry << 7, 0 = no drone) -- in 4 groups of
// lay::code_cpg(W) cells, each padded to code_cpg8 (zero codes), so an act
// kernel lane group reads its group with 16-B loads.  The WindowedGridView
// channels are the same functions of (object, air) the observation writer
// uses (wrappers.py:10-31), so a policy that builds its inputs from the code
// sees the observation's values exactly.  Written by write_obs_wave<CODE>.
template <class GEO>
__device__ __forceinline__ uint16_t* code_row(const StepArgs& a, int64_t wenv0, const GEO& g) {
    return reinterpret_cast<uint16_t*>(a.code) + wenv0 * (int64_t)(4 * lay::code_cpg8((int)g.W()));
}

// drl_step_code_replay: the ring slot of env e's transition (e >= ring_first;
// e - ring_first < ring_cap, so one wrap at most) -- drl_replay_add's ring_slot
template <class A>
__device__ __forceinline__ int64_t step_ring_slot(const A& a, int64_t e) {
    const int64_t s = a.ring_base + (e - a.ring_first);
    return s >= a.ring_cap ? s - a.ring_cap : s;
}

// ... and its code rows: obs = the row the act read (code_prev), next_obs = the
// row this step wrote (still in the wave's LDS staging, `cst`).  Streaming
// stores, as drl_replay_add16_kernel: the ring is read back only by a later
// sample.  VR = 16-B vectors per row; vector v = lane + 64 q of the wave's
// rows (q < RQ) is loaded ahead into pre[q] (step_ring_prefetch), any past
// 64 RQ (runtime windows wider than 9x9) are loaded in the sink.
template <class A>
__device__ __forceinline__ bool ring_vec(const A& a, int64_t wenv0, uint32_t v, uint32_t VR, int64_t* e,
                                         uint32_t* col) {
    const uint32_t el = v / VR;
    *col = v - el * VR;
    *e = wenv0 + el;
    return *e >= a.ring_first;
}

template <int RQ, class A>
__device__ __forceinline__ void step_ring_prefetch(const A& a, int64_t wenv0, int nenv_w, int lane, uint32_t VR,
                                                   u32x4 (&pre)[RQ]) {
    const uint32_t nv = (uint32_t)nenv_w * VR;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
        const uint32_t v = (uint32_t)(lane + 64 * q);
        int64_t e;
        uint32_t col;
        if (v < nv && ring_vec(a, wenv0, v, VR, &e, &col))
            pre[q] = reinterpret_cast<const u32x4*>(a.code_prev)[e * VR + col];
    }
}

// (The rows' scalars -- drone index 0's action, reward and done -- are stored
// where the step writes its rewards, from registers: reading them back here
// behind a workgroup fence measured 0.3 us (C3) and 3.5 us (C5) slower per
// loop step.)
template <int RQ, class A>
__device__ __forceinline__ void step_ring_sink(const A& a, int64_t wenv0, int nenv_w, const l_u16* cst,
                                               int lane, uint32_t VR, const u32x4 (&pre)[RQ]) {
    const l_u4* cv = reinterpret_cast<const l_u4*>(cst);
    const uint32_t nv = (uint32_t)nenv_w * VR;
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
        const uint32_t v = (uint32_t)(lane + 64 * q);
        int64_t e;
        uint32_t col;
        if (v < nv && ring_vec(a, wenv0, v, VR, &e, &col)) {
            const int64_t slot = step_ring_slot(a, e);
            const u32x4 next = cv[v];
            __builtin_nontemporal_store(next, reinterpret_cast<u32x4*>(a.ring_next) + slot * VR + col);
            __builtin_nontemporal_store(pre[q], reinterpret_cast<u32x4*>(a.ring_obs) + slot * VR + col);
        }
    }
    for (uint32_t v = (uint32_t)(lane + 64 * RQ); v < nv; v += 64) {
        int64_t e;
        uint32_t col;
        if (!ring_vec(a, wenv0, v, VR, &e, &col)) continue;
        const int64_t slot = step_ring_slot(a, e);
        const u32x4 prev = reinterpret_cast<const u32x4*>(a.code_prev)[e * VR + col];
        const u32x4 next = cv[v];
        __builtin_nontemporal_store(next, reinterpret_cast<u32x4*>(a.ring_next) + slot * VR + col);
        __builtin_nontemporal_store(prev, reinterpret_cast<u32x4*>(a.ring_obs) + slot * VR + col);
    }
}

// Each drone paints its air byte into every observed window (drone indices
// 0..K-1) that contains it.  posidx must be final.
template <class GEO>
__device__ __forceinline__ void paint_windows(l_u8* paint, const l_u16* posidx, int y, int x, uint8_t airbyte,
                                              const GEO& g) {
    const int W = (int)g.W(), K = g.K(), R = g.radius();
    for (int k = 0; k < K; ++k) {
        const uint32_t pk = posidx[k];
        const int pky = (int)g.div_side(pk);
        const int pkx = (int)pk - pky * g.side();
        const int dy = y - pky + R, dx = x - pkx + R;
        if ((unsigned)dy < (unsigned)W && (unsigned)dx < (unsigned)W) paint[k * W * W + dy * W + dx] = airbyte;
    }
}

__device__ __forceinline__ void chg_push(const WaveLds& w, int grp, int nchg_cap, int cell) {
    const uint32_t q = __atomic_fetch_add(&w.cnt[grp * 4], 1u, __ATOMIC_RELAXED);
    if (q < (uint32_t)nchg_cap) w.chg[grp * nchg_cap + q] = (uint16_t)cell;
}

__device__ __forceinline__ bool bm_test(const l_u32* bm, int cell) { return (bm[cell >> 5] >> (cell & 31)) & 1u; }
__device__ __forceinline__ void bm_set(l_u32* bm, int cell) { __atomic_fetch_or(&bm[cell >> 5], 1u << (cell & 31), __ATOMIC_RELAXED); }

// Group-relative lane masks: 32-bit when a group fits a 32-lane half.
template <int P> struct GMaskT { using type = uint32_t; };  // P <= 32
template <> struct GMaskT<64> { using type = uint64_t; };

template <int P>
__device__ __forceinline__ typename GMaskT<P>::type gballot(bool pred, int gshift) {
    using M = typename GMaskT<P>::type;
    const uint64_t b = __ballot(pred);
    if constexpr (P == 64) return b;
    else return (M)(b >> gshift) & (M)((1ull << P) - 1ull);
}
__device__ __forceinline__ int popc(uint32_t m) { return __popc(m); }
__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ int lobit(uint32_t m) { return __ffs(m) - 1; }
__device__ __forceinline__ int lobit(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }
__device__ __forceinline__ int hibit(uint32_t m) { return 31 - __clz(m); }
__device__ __forceinline__ int hibit(uint64_t m) { return 63 - __clzll((long long)m); }

// __shfl(v, src, P) with the lane id passed in (so a caller can keep the
// address math from being hoisted; see step_batch)
template <int P>
__device__ __forceinline__ int gshfl(int v, int src, int lane) {
#ifdef DRL_HIP_SHFL  // diagnostic A/B: HIP's own __shfl
    return __shfl(v, src, P);
#else
    return __builtin_amdgcn_ds_bpermute(((lane & ~(P - 1)) + (src & (P - 1))) << 2, v);
#endif
}

// The same exchange over a whole group with the source lanes known at compile time: the group's base as a
// bpermute byte address, made opaque where a scan starts (gbase), so each source's address is that base plus
// an immediate offset formed at its use -- not P addresses hoisted to the kernel's start and held live in
// registers across it (at P = 32 that was 32 VGPRs of the C5 step's 114)
template <int P>
__device__ __forceinline__ int gbase(int lane) {
    int b = (lane & ~(P - 1)) << 2;
    asm volatile("" : "+v"(b));
    return b;
}
template <int P>
__device__ __forceinline__ int gshfl_at(int v, int base, int src) {
    return __builtin_amdgcn_ds_bpermute(base + ((src & (P - 1)) << 2), v);
}

// Value of lane (lane ^ K) within each 8-lane group, K = 1..7, by DPP (no LDS
// round trip): quad_perm for K = 1, 2, 3, row_half_mirror (lane i <- 7 - i =
// i ^ 7) for K = 7, and half_mirror after quad_perm(K ^ 7) for K = 4, 5, 6.
template <int K>
__device__ __forceinline__ int xor_lane8(int v) {
    if constexpr (K == 1) return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);       // [1,0,3,2]
    else if constexpr (K == 2) return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
    else if constexpr (K == 3) return __builtin_amdgcn_update_dpp(0, v, 0x1B, 0xf, 0xf, false);  // [3,2,1,0]
    else if constexpr (K == 7) return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);
    else return __builtin_amdgcn_update_dpp(0, xor_lane8<K ^ 7>(v), 0x141, 0xf, 0xf, false);
}
// ... within each 16-lane row, K = 1..15: row_mirror (lane i <- 15 - i = i ^ 15)
// after xor_lane8<K ^ 15> for K >= 8.
template <int K>
__device__ __forceinline__ int xor_lane16(int v) {
    if constexpr (K < 8) return xor_lane8<K>(v);
    else return __builtin_amdgcn_update_dpp(0, xor_lane8<K ^ 15>(v), 0x140, 0xf, 0xf, false);
}
// f(value of lane j ^ k, k) for k = 1..P-1 within P-lane groups (P = 8 or 16)
template <int P, int K = 1, class F>
__device__ __forceinline__ void for_other_lanes(int v, F&& f) {
    if constexpr (K < P) {
        f(P == 8 ? xor_lane8<K>(v) : xor_lane16<K>(v), K);
        for_other_lanes<P, K + 1>(v, f);
    }
}

// ------------------------------------------------------------------ step ---
// One wave per block.  P <= 8 (small grids, LDS <= 5 KB/wave): cap registers
// at 64 so 8 waves fit a SIMD and every wave of a 65536-env C3 launch is
// resident at once (at 6 waves/SIMD a second, tail-heavy generation formed).
// Wider groups are LDS-limited below 8 waves/SIMD: no cap (it only spilled).
// Global addressing: 64-bit wave bases (scalar) + 32-bit lane offsets.
// One batch (the wave's GPW envs starting at wenv0) of the step.  ROLL: a
// rollout of a.steps steps (drl_rollout) with the state kept on chip between
// them -- ground in LDS, drone records in the scratch area (O order) and the
// MT index in a register -- and written back once at the end; the actions of
// step t+1 are loaded during step t.  NT: streaming observation stores.
// CODE: also write drone 0's policy code (a separate instance: the code
// writer's registers would otherwise spill in the plain step at 64 VGPRs).
// RING (with CODE): also land drone 0's transitions in a replay ring
// (drl_step_code_replay, step_ring_sink).
// The synthetic action stream (drl_synth_actions, the oracle's synth_actions): drone `drone` of global env
// `genv` at (seed, step) -- a counter hash, so any kernel can draw any element.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ int synth_action(uint64_t seed, uint64_t step, uint64_t genv, uint64_t drone) {
    const uint64_t h = splitmix64(seed ^ splitmix64((step << 40) ^ (genv << 8) ^ drone));
    return (int)(((h >> 32) * 5ull) >> 32);
}

template <int P, class GEO, bool ROLL, bool NT, bool CODE = false, bool RING = false>
__device__ __forceinline__ void step_batch(const StepArgs& a, int64_t wenv0) {
    using GMask = typename GMaskT<P>::type;
    constexpr int GPW = 64 / P;
    static_assert(!ROLL || P >= kRolloutNoObsMinLanes, "narrow groups roll out as drl_step launches");
    constexpr int D = step_draws(P);             // draws per lane per dry-ring respawn round
    constexpr int QL = step_cq(P);               // ring entries per lane per batch
    using CM = typename GMaskT<(P * D <= 32 ? 32 : 64)>::type;  // round-position masks
#ifndef DRL_SHFL_BATCH
#define DRL_SHFL_BATCH 16
#endif
    constexpr int CH = P < DRL_SHFL_BATCH ? P : DRL_SHFL_BATCH;  // shuffle batch
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
    // this wave's LDS image (workgroups of one wave, or of step_wpb(P) waves: see drl_step_kernel)
    unsigned char* const smem = smem_all + (size_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) *
                                               (size_t)((a.wave_lds + 15) & ~15);
    const GEO g{a};
    const int lane0 = threadIdx.x & 63;
    const int grp0 = lane0 / P;
    const int j0 = lane0 % P;
    const int nenv_w = (int)min((int64_t)GPW, a.E - wenv0);
    if (nenv_w <= 0) return;
    const bool env_ok0 = grp0 < nenv_w;
    const int G = g.side(), N = g.n(), gstride = g.gstride(), nchg = g.nchg();
    const WaveLds W = carve((l_u8*)smem, GPW, P, g);
    // the wave's slices of the state (scalar bases)
    uint32_t* const drones_w = a.drones + wenv0 * N;
    uint32_t* const mt_w = a.mt + wenv0 * MT_WORDS;
    const int pstride = g.pstride();
    uint8_t* const ground_w = a.ground + wenv0 * pstride;  // packed rows
    const uint32_t rl0 = (uint32_t)(grp0 * N);  // lane's env offset in [env][drone] arrays of the wave

    DRL_STAMP(0);
    // ---- loads, in one round trip: the env's mt_index word (one load per
    // lane, all lanes of a group at one address), then the LDS zeroing (LDS
    // writes must precede the LDS-DMA or they wait for it), the drone record
    // and the action of drone index j, the ground by LDS-DMA.  Consumers of
    // the ground come after the claims scan.
    uint32_t mi[GPW];  // uniform addresses, nothing written before: scalar loads (lgkmcnt)
#pragma unroll
    for (int e = 0; e < GPW; ++e) mi[e] = a.mt_index[wenv0 + min(e, nenv_w - 1)];
    lds_zero(W.bm, GPW * g.lds_bm(), lane0);
    if (GEO::kObs && (a.obs || CODE)) lds_zero(W.paint, GPW * g.lds_paint(), lane0);
    if (lane0 < GPW) W.cnt[lane0 * 4] = 0u;
    wave_sync();
    const bool active0 = env_ok0 && j0 < N;
    // unconditional loads at clamped indices (no exec-mask branches around
    // them, so the wait counts stay exact); inactive lanes discard the values
    const uint32_t li0 = min(rl0 + (uint32_t)j0, (uint32_t)(nenv_w * N - 1));
    const uint32_t rec_ld = drones_w[li0];
#ifdef DRL_DIAG_ACT_U8  // bytes-only diagnostic build (wrong actions): one byte per action
    const int act_ld = reinterpret_cast<const uint8_t*>(a.actions)[wenv0 * N + li0] % 5;
#else
    // (drl_step_code_replay_synth: column 0 only; drone indices >= 1 take the counter hash below)
    const int act_ld = a.actions[(RING && a.synth) ? (wenv0 + min(grp0, nenv_w - 1)) * (int64_t)N
                                                   : wenv0 * N + li0];
#endif
    // the packed grounds: loaded now, unpacked into LDS after the claim scan (compile-time geometry)
    [[maybe_unused]] NibStage<(GEO::kPstride > 0 ? GPW * GEO::kPstride / 16 : 1), (GEO::kGstride == GEO::kPstride)> nib;
    if constexpr (GEO::kPstride > 0) nib.load(ground_w, nenv_w * pstride, lane0);
    else stage_ground_nib(ground_w, nenv_w * pstride, W.gl, lane0, g.nib());
    __builtin_amdgcn_sched_barrier(0);  // issue every load above before waiting for the MT index
    // the synthetic actions of drone indices >= 1 (drl_step_code_replay_synth), while the loads are in flight
    [[maybe_unused]] int syn_act = 0;
    if constexpr (RING) {
        if (a.synth) syn_act = synth_action(a.synth_seed, a.synth_step, (uint64_t)(a.env_offset + wenv0 + grp0),
                                            (uint64_t)j0);
    }
    uint32_t mword = mi[0];  // the env's mt_index word: index, block, ring head / count
#pragma unroll
    for (int e = 1; e < GPW; ++e) mword = (grp0 >= e) ? mi[e] : mword;
    uint32_t rec = active0 ? rec_ld : 0u;
    int my_action = active0 ? act_ld : 4;
    if constexpr (RING) {
        if (a.synth && j0 != 0 && active0) my_action = syn_act;
    }
    if (!env_ok0) mword = (uint32_t)MT_N;
    // the stream position is read only after the ring's entries (they carry
    // it along), so nothing holds it across the claim phase; a rollout keeps
    // the word (index, block, ring head / count) in a register between steps
    int midx = 0;
    l_u32* const stash = W.stash;  // ROLL: records between steps ([GPW][P], O order)
    // drl_rollout takes the rings' entries while they last, then draws from
    // the stream, at 16 <= P <= DRL_ROLL_RING_MAXP (16).  Other groups discard the
    // entries instead (they are a cache of the same draws; the refill at the
    // end rebuilds them), which frees the ring code's registers: C5's rollout
    // runs 3 waves per SIMD with it (126 -> 138 VGPRs) and measured 134 us/step
    // against 119 without; C4's gains from the entries (27.95 vs 29.2).
    constexpr bool kRing = !ROLL || (DRL_ROLL_RING && P >= kRolloutMinLanes && P <= DRL_ROLL_RING_MAXP);
    uint32_t cq[QL];  // the step's ring entries
    auto ring_issue = [&](const uint32_t mw) __attribute__((always_inline)) {
        const uint32_t rbase = (uint32_t)(env_ok0 ? grp0 : 0) * MT_WORDS + MT_RING;
        const int qh = mi_head(mw);
#pragma unroll
#ifdef DRL_DIAG_RING_FIXED  // bytes-only diagnostic build (wrong results): every env reads the wave's first window
        for (int r = 0; r < QL; ++r) cq[r] = mt_w[MT_RING + ((j0 + P * r) & (CAND_Q - 1))];
#else
        for (int r = 0; r < QL; ++r) cq[r] = mt_w[rbase + ((qh + j0 + P * r) & (CAND_Q - 1))];
#endif
    };
    int act_next = 4;
    const int T = ROLL ? a.steps : 1;
    for (int t = 0; t < T; ++t) {
    const int lane = lane0, grp = lane / P, j = lane % P;
    const bool env_ok = grp < nenv_w;
    const bool active = env_ok && j < N;
    const uint32_t rl = (uint32_t)(grp * N);
    const uint32_t li = min(rl + (uint32_t)j, (uint32_t)(nenv_w * N - 1));
    l_u8* gl = W.gl + grp * gstride;
    l_u32* bm = W.bm + grp * (g.lds_bm() / 4);
    l_u16* posidx = W.posidx + grp * g.np();
    const uint32_t* mrow = mt_w + (uint32_t)(env_ok ? grp : 0) * MT_WORDS;  // drl_step: set after the ring
    if constexpr (ROLL) {
        if (t > 0) {  // the previous step left its records in the stash
            rec = active ? stash[lane] : 0u;
            my_action = active ? act_next : 4;
            wave_sync();
            lds_zero(W.bm, GPW * g.lds_bm(), lane);
            if (GEO::kObs && a.obs) lds_zero(W.paint, GPW * g.lds_paint(), lane);
            wave_sync();
        }
        if (t + 1 < T) act_next = a.actions[(t + 1) * a.act_tstride + wenv0 * N + li];
    }

#ifdef DRL_NIB_EARLY  // (A/B: a packed LDS image stored before the claim scan, its registers freed)
    if constexpr (GEO::kGstride > 0 && !ROLL) {
        if (g.nib()) nib.store(W.gl, lane0, true);
    }
#endif
    DRL_STAMP(1);
    const int y = rec & 255u, x = (rec >> 8) & 255u;
    const int idx = ((int)(rec >> 25) < N) ? (int)(rec >> 25) : j;  // corrupt records never index out of bounds
    int c = (rec >> 16) & 255u;
    int carry = (rec >> 24) & 1u;
    int act;  // actions are by drone index (env.py:125)
    act = gshfl<P>(my_action, idx, lane);
    // The env's next P*QL ring entries (drl_refill drew them ahead), issued
    // once the records have landed (LDS-DMA makes the compiler wait for every
    // outstanding load before the first record use), so their latency
    // overlaps the claim / effect / ordering phases.  MT words are read only
    // if the ring runs dry.
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kRing) ring_issue(mword);
    // once a rollout's ring is empty (or discarded), the first respawn
    // round's MT words are loaded here too, so the stream draws do not start
    // with a round trip
    [[maybe_unused]] uint32_t pfq[ROLL ? D : 1];
    [[maybe_unused]] bool pf_live = false;
    if constexpr (ROLL) {
        pf_live = (!kRing || mi_cnt(mword) == 0) && mi_idx(mword) + D * P <= MT_N;
        const uint32_t* src = mt_w + (uint32_t)(env_ok ? grp : 0) * MT_WORDS + (uint32_t)mi_par(mword) * MT_ALT;
#pragma unroll
        for (int q = 0; q < D; ++q) pfq[q] = load_l2(src + min(mi_idx(mword) + q * P + j, MT_N - 1));
    }
    __builtin_amdgcn_sched_barrier(0);
    if (active) {
        if (act < 0) act += 5;  // Python negative list index
        if ((unsigned)act > 4u) {
            if (a.err) atomicOr(a.err, DRL_ERR_BAD_ACTION);
            act = 4;
        }
    }
    // ACTION_TO_DIRECTION (env.py:26): LEFT(0,-1) DOWN(1,0) RIGHT(0,1) UP(-1,0) STAY(0,0)
    const int ty = y + (act == 1) - (act == 3);
    const int tx = x + (act == 2) - (act == 0);
    const bool inb = active && ty >= 0 && ty < G && tx >= 0 && tx < G;
    const int tcell = inb ? ty * G + tx : -1 - j;  // unique negatives never match

    // ---- phase 1 claims (env.py:124-140): first in O order claims a cell;
    // later ones crash (list A) and record the cell; OOB crashes (list A).
    bool earlier = false;
    int later_min = P;
    if constexpr ((P == 8 || P == 16) && DRL_DPP8) {  // the group's other targets by DPP
        for_other_lanes<P>(tcell, [&](int o, int k) {
            const int s = j ^ k;
            const bool same = o == tcell;
            earlier |= same && s < j;
            later_min = (same && s > j && s < later_min) ? s : later_min;
        });
    } else {
    const int gb = gbase<P>(lane);
#pragma unroll
    for (int s0 = 0; s0 < P; s0 += CH) {
        int ts[CH];
#pragma unroll
        for (int t = 0; t < CH; ++t) ts[t] = gshfl_at<P>(tcell, gb, s0 + t);
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const int s = s0 + t;
            const bool same = ts[t] == tcell;
            earlier |= same && s < j;
            later_min = (same && s > j && s < later_min) ? s : later_min;
        }
    }
    }
    const bool claimer = inb && !earlier;
    const bool crashA = active && !claimer;
    if constexpr (GEO::kGstride > 0) {
#ifdef DRL_NIB_EARLY
        if (t == 0 && (ROLL || !g.nib())) nib.store(W.gl, lane0, g.nib());
#else
        if (t == 0) nib.store(W.gl, lane0, g.nib());  // (a rollout stages once)
#endif
    }
    // the grounds are in LDS; wave_sync orders lanes
    wave_sync();

    DRL_STAMP(2);
    // ---- phase 2 effects on claimers (env.py:143-172), own cell only
    float reward = 0.0f;
    bool dead = false, deliver = false;
    if (claimer) {
        const int obj = gl_get(g, gl, tcell);
        if (obj == OBJ_STATION) {
            c = min(100, c + a.charge);
            reward = a.r_charge;
        } else {
            c -= a.discharge;
            dead = c <= 0;
        }
        if (obj == OBJ_PACKET && !carry) {
            reward = a.r_pickup;
            carry = 1;
            gl_clear(g, gl, tcell);
            if constexpr (!ROLL) chg_push(W, grp, nchg, tcell);
        } else if (obj == OBJ_DROPZONE && carry) {
            reward = a.r_delivery;
            carry = 0;
            gl_clear(g, gl, tcell);
            deliver = true;
            if constexpr (!ROLL) chg_push(W, grp, nchg, tcell);
        }
        if (obj == OBJ_SKYSCRAPER) dead = true;
    }

    // ---- phase 3/4 ordering (env.py:177-195): crash list B = claimers at a
    // collision cell (ordered by the cell's first second-comer) then battery /
    // skyscraper deaths (claimer order).  New order O' = survivors, A, B.
    const bool collided = claimer && later_min < P;
    const bool crashB = claimer && (collided || dead);
    const bool survivor = claimer && !crashB;
    const bool crashed = crashA || crashB;
    const int gshift = grp * P;
    const uint64_t gm = (P == 64) ? ~0ull : (((1ull << (P & 63)) - 1ull) << gshift);
    const uint64_t lower = (1ull << lane) - 1ull;
    const uint64_t bS = __ballot(survivor) & gm;
    const uint64_t bA = __ballot(crashA) & gm;
    const uint64_t bB = __ballot(crashB) & gm;
    const int nS = __popcll(bS), nA = __popcll(bA), nR = nA + __popcll(bB);
    int rankB = 0;
    if (__ballot(crashB)) {
        const int bkey = crashB ? (collided ? later_min : P + j) : 4 * P;
        if constexpr ((P == 8 || P == 16) && DRL_DPP8) {
            for_other_lanes<P>(bkey, [&](int o, int) { rankB += o < bkey; });
        } else {
        const int gb = gbase<P>(lane);
#pragma unroll
        for (int s0 = 0; s0 < P; s0 += CH) {
            int ks[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) ks[t] = gshfl_at<P>(bkey, gb, s0 + t);
#pragma unroll
            for (int t = 0; t < CH; ++t) rankB += (ks[t] < bkey);
        }
        }
    }
    const int newslot = survivor ? __popcll(bS & lower)
                                 : (crashA ? nS + __popcll(bA & lower) : (crashB ? nS + nA + rankB : j));
    const int n_deliver = __popcll(__ballot(deliver) & gm);
    const int n_pack = n_deliver + __popcll(__ballot(crashed && carry) & gm);
    const int total = nR + n_pack + n_deliver;
    if (crashed) {
        c = 100;
        carry = 0;
        reward = a.r_crash;
    }
    int pos = survivor ? tcell : -1;
    if (survivor) bm_set(bm, tcell);
    wave_sync();

    DRL_STAMP(3);
    // ---- respawns (env.py:186-210, _find_respawn_position :226-233):
    // items w < nR: crashed drones (mask: drones | skyscrapers); then n_pack
    // packets, then n_deliver dropzones (mask: any ground object).  Each round
    // draws D*P consecutive MT outputs, keeps those < side (randint(0, side-1)
    // == _randbelow(side)) and pairs accepted draws as (y, x).  A placement
    // always ends on the second draw of a pair, so the pairing is the same for
    // every item: the round's candidate cells are read from LDS once and
    // several items are placed per round, later items seeing the cells placed
    // earlier in the round through register compares.
#ifdef DRL_DIAG_NO_RESPAWN  // timing-only diagnostic build (wrong results): the step without its respawn rounds
    int w = total, have_y = 0, yv = 0;
#else
    int w = 0, have_y = 0, yv = 0;
#endif
    const int shift = 32 - g.kbits();
    const int my_item = crashed ? newslot - nS : -1;  // this drone's respawn item
    {
        // ---- fast path: the ring's candidate cells, i.e. the
        // stream's next accepted (y, x) pairs, P per batch, one per lane.  An
        // item takes the first candidate after the previous item's that is free
        // under its mask, so the items of one class (drones: drones |
        // skyscrapers; packets, then dropzones: any ground object) are the
        // class's first free candidates that do not repeat an earlier candidate
        // of the class (a repeat is either occupied or the cell an earlier item
        // took).  One ballot and a rank place a whole class; the next class
        // starts after its last item.  Earlier batches' placements are in the
        // bitmap / ground.
        const int qcnt = (kRing && env_ok) ? mi_cnt(mword) : 0;
        const int GGc = G * G;
        int start = 0;          // ring entries consumed (group-uniform)
        uint32_t ent_last = 0;  // the last consumed entry (group-uniform)
        auto batch = [&](const uint32_t cqr, const int r) __attribute__((always_inline)) {
            const int cell = ce_cell(cqr);
            const bool valid = env_ok && P * r + j < qcnt && cell < GGc;
            const int ccell = valid ? cell : 0;
            const int tg = valid ? cell : -1 - j;  // unique negatives never match
            int prev = -1;                        // nearest earlier lane of the batch with the same cell
            if constexpr ((P == 8 || P == 16) && DRL_DPP8) {
                for_other_lanes<P>(tg, [&](int o, int k) {
                    const int s2 = j ^ k;
                    prev = (o == tg && s2 < j && s2 > prev) ? s2 : prev;
                });
            } else {
                const int gb = gbase<P>(lane);
#pragma unroll
                for (int s0 = 0; s0 < P; s0 += CH) {
                    int ts[CH];
#pragma unroll
                    for (int t2 = 0; t2 < CH; ++t2) ts[t2] = gshfl_at<P>(tg, gb, s0 + t2);
#pragma unroll
                    for (int t2 = 0; t2 < CH; ++t2) prev = (ts[t2] == tg && s0 + t2 < j) ? s0 + t2 : prev;
                }
            }
            const int gobj = gl_get(g, gl, ccell);
            const bool occ = bm_test(bm, ccell);
            const int bend = min(P * (r + 1), qcnt);  // end of the batch's valid entries
#pragma unroll
            for (int cs = 0; cs < 3; ++cs) {  // class steps: drones, packets, dropzones
                const bool act = env_ok && w < total && start < bend;
                if (!__ballot(act)) break;
                const bool isd = w < nR;
                const int cls_end = isd ? nR : (w < nR + n_pack ? nR + n_pack : total);
                const int need = cls_end - w;
                const int gnow = cs == 0 ? gobj : gl_get(g, gl, ccell);  // packets placed by the previous step
                const bool fresh = valid && P * r + j >= start && (prev < 0 || P * r + prev < start);
                const bool ok = act && fresh && (isd ? (!occ && gnow != OBJ_SKYSCRAPER) : gnow == OBJ_EMPTY);
                const GMask M = gballot<P>(ok, gshift);
                const int k = min(popc(M), need);
                const int rank = popc(M & ((GMask(1) << j) - GMask(1)));
                const bool chosen = ok && rank < k;
                const GMask C = gballot<P>(chosen, gshift);
                if (chosen) {
                    if (isd) {
                        posidx[w + rank] = (uint16_t)cell;  // item slot (posidx is rewritten at write-back)
                        bm_set(bm, cell);
                    } else {
                        gl_put(g, gl, cell, (w + rank < nR + n_pack) ? OBJ_PACKET : OBJ_DROPZONE);
                        if constexpr (!ROLL) chg_push(W, grp, nchg, cell);
                    }
                }
                // the class ends at its last item, or takes the rest of the batch
                const bool done = k == need;
                const uint32_t el = (uint32_t)gshfl<P>((int)cqr, done ? hibit(C) : bend - 1 - P * r, lane);
                if (act) {
                    start = done ? P * r + hibit(C) + 1 : bend;
                    ent_last = el;
                    w += k;
                }
                wave_sync();
            }
        };
        if constexpr (kRing) {
#pragma unroll
            for (int r = 0; r < QL; ++r) {
                if (!__ballot(env_ok && w < total && start < qcnt)) break;
                batch(cq[r], r);
            }
            // rare: more candidates than the lanes hold (e.g. many crashes at once):
            // the ring's next entries, one more round trip per batch
            for (int r = QL; r < CAND_Q / P; ++r) {
                if (!__ballot(env_ok && w < total && start < qcnt)) break;
                const uint32_t* ring = mt_w + (uint32_t)(env_ok ? grp : 0) * MT_WORDS + MT_RING;
                batch(ring[(mi_head(mword) + j + P * r) & (CAND_Q - 1)], r);
            }
        }
        if (crashed && my_item < w) pos = posidx[my_item];
        // stream position after the consumed entries; a dry ring continues from
        // the end of its last entry
        const bool dry = env_ok && w < total;  // (the ring's loaded entries are used up)
        const int ncons = start;
        const uint32_t ent = ent_last;
        midx = min(ncons > 0 ? ce_idx(ent) : mi_idx(mword), MT_N);
        const int mpar = ncons > 0 ? ce_par(ent) : mi_par(mword);
        // the ring served every item: the new word waits in LDS until the
        // write-back (a global store now would hold the first later vmcnt
        // wait); a dry ring's is made after the draws below
        const uint32_t nword = mi_pack(midx, mpar, (mi_head(mword) + ncons) & (CAND_Q - 1), qcnt - ncons);
        if constexpr (ROLL) {
            if (!dry) mword = nword;
        } else if (env_ok && j == 0 && !dry) {
            W.cnt[grp * 4 + 1] = nword;
        }
        mrow += (uint32_t)mpar * MT_ALT;
        wave_sync();
    }
    uint32_t rounds = 0;
    [[maybe_unused]] uint32_t rounds_w = 0;  // wave-level loop trips (diagnostics)
    [[maybe_unused]] unsigned long long sub_t0 = 0, sub_t1 = 0, sub_t2 = 0, sub_t3 = 0, sub_acc[4] = {0, 0, 0, 0};
    for (;;) {
        const bool work = env_ok && w < total;
        if (!__ballot(work)) break;
        ++rounds_w;
        DRL_SUBT(sub_t0);
        uint64_t need = __ballot(work && j == 0 && midx >= MT_N);
        while (need) {
            const int tl = __ffsll((unsigned long long)need) - 1;
            need &= need - 1ull;
#ifndef DRL_DIAG_NO_TWIST  // timing-only builds (wrong streams)
            {  // lane tl's stream block (either)
                const uint64_t pr = (uint64_t)(uintptr_t)mrow;
                const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pr, tl);
                const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pr >> 32), tl);
                twist_wave(reinterpret_cast<uint32_t*>((hi << 32) | lo), lane);
            }
#endif
            if (grp == tl / P) midx = 0;
        }
        // ---- one round: D*P consecutive draws of this env's stream; position
        // d = q*P + j is lane j's q-th draw (branch-free; groups without work
        // compute and discard)
        DRL_SUBT(sub_t1);
        const int avail = MT_N - midx;
        int rq[D], ccq[D];
        bool candq[D], accq[D];
        GMask mq[D];
        CM accall = 0;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const int d = q * P + j;
            const bool valid = work && d < avail;
            uint32_t word = 0u;
            if constexpr (ROLL) word = pfq[q];  // (pf_live: the same words)
            if (__ballot(valid && !pf_live)) word = (valid && !pf_live) ? load_l2(mrow + midx + d) : word;
            rq[q] = valid ? (int)(temper(word) >> shift) : G;
            accq[q] = rq[q] < G;
            mq[q] = gballot<P>(accq[q], gshift);
            accall |= CM(mq[q]) << (q * P);
        }
        // value r at a round position (group-uniform b)
        auto r_at = [&](int b) {
            int v = gshfl<P>(rq[0], b % P, lane);
#pragma unroll
            for (int q = 1; q < D; ++q) {
                const int vq = gshfl<P>(rq[q], b % P, lane);
                v = (b / P == q) ? vq : v;
            }
            return v;
        };
        GMask okd = 0, okg = 0;
        CM okdc = 0, okgc = 0;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const CM prevm = accall & ((CM(1) << (q * P + j)) - CM(1));
            const int apos = have_y + popc(prevm);
            const int pl = prevm ? hibit(prevm) : 0;
            const int rp = r_at(pl);
            const int ycand = prevm ? rp : yv;
            candq[q] = accq[q] && (apos & 1);
            ccq[q] = candq[q] ? ycand * G + rq[q] : 0;
            const int gobj = gl_get(g, gl, ccq[q]);
            const bool occ = bm_test(bm, ccq[q]);
            okd = gballot<P>(candq[q] && !occ && gobj != OBJ_SKYSCRAPER, gshift);  // drone items
            okg = gballot<P>(candq[q] && gobj == OBJ_EMPTY, gshift);              // packet / dropzone items
            okdc |= CM(okd) << (q * P);
            okgc |= CM(okg) << (q * P);
        }
        DRL_SUBT(sub_t2);
        // ---- place as many items as this round's candidates allow: a placement
        // ends on a pair's second draw, so the pairing holds for the next item;
        // cells placed this round are removed from the masks by compare-ballots.
        int last = -1;
        bool more = work;
#ifdef DRL_DIAG_NO_PLACE  // timing-only (wrong results): every item placed at once at the first candidate
        if (more) {
            const CM m0 = (w < nR ? okdc : okgc);
            last = m0 ? lobit(m0) : D * P - 1;
            pos = (my_item >= 0 && m0) ? ccq[0] : pos;
            w = m0 ? total : w;
            more = false;
        }
#endif
        while (__ballot(more)) {
            if (more) {
                const bool isd = w < nR;
                const CM after = (last < 0) ? ~CM(0) : ~((CM(2) << last) - CM(1));
                const CM m = (isd ? okdc : okgc) & after;
                if (!m) {
                    more = false;
                } else {
                    const int b = lobit(m);
                    int cell = gshfl<P>(ccq[0], b % P, lane);
#pragma unroll
                    for (int q = 1; q < D; ++q) {
                        const int cq = gshfl<P>(ccq[q], b % P, lane);
                        cell = (b / P == q) ? cq : cell;
                    }
                    CM same = 0;
#pragma unroll
                    for (int q = 0; q < D; ++q) same |= CM(gballot<P>(candq[q] && ccq[q] == cell, gshift)) << (q * P);
                    if (isd) {
                        pos = (my_item == w) ? cell : pos;
                        if (j == 0) bm_set(bm, cell);
                        okdc &= ~same;
                    } else {
                        if (j == 0) {
                            gl_put(g, gl, cell, (w < nR + n_pack) ? OBJ_PACKET : OBJ_DROPZONE);
                            if constexpr (!ROLL) chg_push(W, grp, nchg, cell);
                        }
                        okgc &= ~same;
                    }
                    last = b;
                    ++w;
                    more = w < total;
                }
            }
        }
        DRL_SUBT(sub_t3);
        if constexpr (ROLL) pf_live = false;
        if (work) {
            if (w >= total) {
                midx += last + 1;  // draws after the last placement stay unconsumed
                have_y = 0;
            } else {
                const int cnt = have_y + popc(accall);
                const int yl = r_at(accall ? hibit(accall) : 0);
                if (accall && (cnt & 1)) yv = yl;
                have_y = cnt & 1;
                midx += min(D * P, avail);
            }
            if (++rounds > a.max_rounds) {  // full grid: the reference spins forever
                if (j == 0 && a.err) atomicOr(a.err, DRL_ERR_NO_FREE_CELL);
                w = total;
                if (crashed && pos < 0) pos = 0;
            }
        }
        wave_sync();
#ifdef DRL_STAMPS
        {  // twists | candidates (draws, pairing, masks) | placement | round tail
            unsigned long long t4;
            DRL_SUBT(t4);
            sub_acc[3] += t4 - sub_t3;
        }
        sub_acc[0] += sub_t1 - sub_t0;
        sub_acc[1] += sub_t2 - sub_t1;
        sub_acc[2] += sub_t3 - sub_t2;
#endif
    }
#ifdef DRL_STAMPS
    if (lane == 0)
        for (int k = 0; k < 4; ++k)
            if (g_stamps) g_stamps[((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + 10 + k] = sub_acc[k];
#endif

    DRL_STAMP(4);
#ifdef DRL_STAMPS
    if (lane == 0 && g_stamps) g_stamps[((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + 7] = __builtin_amdgcn_readfirstlane(rounds_w);
#endif
    // ---- _pick_packets_after_respawn (env.py:217-224): distinct cells, parallel
    if (active && pos < 0) pos = 0;  // unreachable for valid params (respawn always finds a cell)
    if (active && !carry && gl_get(g, gl, pos) == OBJ_PACKET) {
        carry = 1;
        gl_clear(g, gl, pos);
        if constexpr (!ROLL) chg_push(W, grp, nchg, pos);
    }

    // ---- write back: records permuted to O', rewards/dones by drone index,
    // changed ground cells as bytes
    const uint32_t py = g.div_side((uint32_t)(pos > 0 ? pos : 0));
    const uint32_t px = (uint32_t)(pos > 0 ? pos : 0) - py * (uint32_t)G;
    const uint32_t rec_out = pack_drone((int)py, (int)px, c, carry, idx);
    // dones: byte stores make the L2 fetch the 128-B line they land in (PMC:
    // ~16 B of reads per env-step at C3); when n_drones % 4 == 0 each env's
    // flags are gathered by drone index in LDS (the occupancy bitmap is dead
    // now) and written as dwords instead
    const bool dpack = a.dones_packed;
    l_u8* const dn = reinterpret_cast<l_u8*>(bm);
    if (active) {
        if constexpr (!ROLL) drones_w[rl + newslot] = rec_out;
        a.rewards[t * a.out_tstride + wenv0 * N + (rl + idx)] = reward;
        if constexpr (RING) {  // drl_step_code_replay: drone index 0's action / reward / done (step_ring_sink)
            const StepArgs& ka = *(const StepArgs*)__builtin_amdgcn_kernarg_segment_ptr();
            const int64_t e = wenv0 + grp;
            if (idx == 0 && e >= ka.ring_first) {
                const int64_t slot = step_ring_slot(ka, e);
                ka.ring_act[slot] = ka.actions[e * N];
                ka.ring_rew[slot] = reward;
                ka.ring_done[slot] = crashed ? 1 : 0;
            }
        }
#ifndef DRL_DIAG_NO_SMALL_WB  // bytes-only diagnostic build: no sub-line stores (dones, mt_index)
        if (dpack) dn[idx] = crashed ? 1 : 0;
        else a.dones[t * a.out_tstride + wenv0 * N + (rl + idx)] = crashed ? 1 : 0;
#endif
        posidx[idx] = (uint16_t)pos;
    }
    if constexpr (ROLL) {  // a dry ring: the stream position after the draws, an empty ring
        if (rounds > 0) mword = mi_pack(midx, mrow != mt_w + (uint32_t)(env_ok ? grp : 0) * MT_WORDS ? 1 : 0, 0, 0);
    } else if (env_ok && j == 0) {
#ifdef DRL_DIAG_NO_SMALL_WB
        if (a.E < 0)
#endif
        a.mt_index[wenv0 + grp] = rounds > 0 ? mi_pack(midx, mrow != mt_w + (uint32_t)grp * MT_WORDS ? 1 : 0, 0, 0)
                                             : W.cnt[grp * 4 + 1];
    }
    wave_sync();
    if (dpack && env_ok && j < (N >> 2))
        reinterpret_cast<uint32_t*>(a.dones + t * a.out_tstride + wenv0 * N + rl)[j] =
            reinterpret_cast<const l_u32*>(dn)[j];
    if (!ROLL && env_ok) {
        const uint32_t nc = W.cnt[grp * 4];
        const l_u16* ch = W.chg + grp * nchg;
        uint8_t* gdst = ground_w + (uint32_t)(grp * pstride);
        // Changes per step <= 4N (N pickups/deliveries, 2N respawned packets and
        // dropzones, N pick-after-respawn) < the list's 6N + 2 entries, so the
        // list never overflows (chg_push drops past capacity regardless).  The
        // loop usually runs once: keep it rolled, unrolled/vectorised copies
        // cost registers the whole kernel pays for.
#ifndef DRL_DIAG_NO_GROUND_WB  // bytes-only diagnostic build (wrong state): no changed-cell write-back
#pragma clang loop unroll(disable) vectorize(disable)
        for (uint32_t q = j; q < min(nc, (uint32_t)nchg); q += P) {  // the cell's packed byte (both nibbles)
            const uint32_t e = ch[q] & ~1u;
            gdst[e >> 1] = g.nib() ? gl[e >> 1] : (uint8_t)(gl[e] | (gl[e + 1] << 4));
        }
#endif
    }
    DRL_STAMP(5);
    if (GEO::kObs && (a.obs || (CODE && !ROLL))) {
        // drl_step_code_replay: the arguments read where they are used (the kernarg segment), so the ring's
        // pointers hold no registers through the step; the transitions' obs rows (code_prev) are loaded
        // before the code is built, so their latency overlaps it
        const StepArgs& ka = *(const StepArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        constexpr int RQ = RING ? (GPW * (GEO::kW > 1 ? lay::code_cpg8((int)GEO::kW) / 2 : 12) + 63) / 64 : 1;
        const uint32_t VR = (uint32_t)lay::code_cpg8((int)g.W()) / 2u;
        [[maybe_unused]] u32x4 rpre[RQ];
        if constexpr (RING) step_ring_prefetch<RQ>(ka, wenv0, nenv_w, lane, VR, rpre);
        if (active) paint_windows(W.paint + grp * g.lds_paint(), posidx, (int)py, (int)px,
                                  (uint8_t)((c + 1) | (carry << 7)), g);
        wave_sync();
        float* obase = a.obs + t * a.obs_tstride + wenv0 * (int64_t)(6u * g.env_cells());
        if constexpr (CODE && !ROLL) {
            uint16_t* crow = code_row(a, wenv0, g);
            l_u16* cst = reinterpret_cast<l_u16*>((l_u8*)smem + a.code_lds);
            if (a.obs) write_obs_wave<NT, true, true>(obase, nenv_w, g, W, a.obs_wide, lane, crow, cst);
            else write_obs_wave<NT, true, false>(obase, nenv_w, g, W, a.obs_wide, lane, crow, cst);
            if constexpr (RING) step_ring_sink<RQ>(ka, wenv0, nenv_w, cst, lane, VR, rpre);
        } else {
            write_obs_wave<NT>(obase, nenv_w, g, W, a.obs_wide, lane);
        }
    }
    DRL_STAMP(6);
    if constexpr (ROLL) {  // records to the stash (the observation stage aliased it until here)
        wave_sync();
        if (active) stash[grp * P + newslot] = rec_out;
    }
    }  // steps
    if constexpr (ROLL) {  // write the state back once: records, MT index, whole grounds
        wave_sync();
        if (active0) drones_w[rl0 + j0] = stash[lane0];
        if (env_ok0 && j0 == 0) a.mt_index[wenv0 + grp0] = mword;
        uint4* dst = reinterpret_cast<uint4*>(ground_w);
        for (int v = lane0; v < nenv_w * pstride / 16; v += 64) {
            if (g.nib()) {
                const u32x4 x = reinterpret_cast<const l_u4*>(W.gl)[v];
                dst[v] = make_uint4(x[0], x[1], x[2], x[3]);
            } else {
                dst[v] = nib_pack_load(W.gl + v * 32);
            }
        }
    }
}

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): the
// blocks that share an XCD (the same blockIdx % 8) take consecutive batches of
// envs, so the lines that neighbouring waves share -- the mt_index words (32
// envs per 128-B line), dones, the observation's boundary lines -- are
// written and re-read in one L2 instead of being filled into up to eight.
// Placement never affects results.  Measured and OFF by default (A/B on one
// box, two rounds each): C3 21.56 vs 21.56 us/step, C5 155.3 vs 151.5 (worse),
// refill 50.0 vs 48.5 us; the step's PMC read bytes fell only 1.5 %.  Build
// with -DDRL_XCD_REMAP=1 to turn it on.
#ifndef DRL_XCD_REMAP
#define DRL_XCD_REMAP 0
#endif
__device__ __forceinline__ uint32_t xcd_block(uint32_t orig, uint32_t n) {
    if (!DRL_XCD_REMAP) return orig;
    const uint32_t q = n / 8, r = n % 8, x = orig % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
}

// One wave per batch of GPW envs.  (Persistent waves looping over 2-4 batches
// were measured slower at C3/C4/C5: halving the resident waves costs more
// latency hiding than the longer waves gain in balance.)
// NT: streaming observation stores (DRL_STEP_OBS_STREAM).  CODE: with the
// policy code (drl_step_code).
// RING: drl_step_code_replay (its own instance: the sink costs the plain
// step's register allocation spills).
// (DRL_STEP_WAVES_P16 / _P32: the register budget of the 16- / 32-lane (C4 / C5) instances as waves per
// SIMD; 1 = no cap)
#ifndef DRL_STEP_WAVES_P16
#define DRL_STEP_WAVES_P16 6  // C4: 43.2 -> 41.2 us per step (profiles/r06_occupancy)
#endif
#ifndef DRL_STEP_WAVES_P32
#define DRL_STEP_WAVES_P32 1
#endif
// (DRL_STEP_WPB_P16 / _P32: waves per workgroup of the 16- / 32-lane instances, each wave its own batch and
// LDS image, no workgroup barrier; 1 = one-wave workgroups)
#ifndef DRL_STEP_WPB_P16
#define DRL_STEP_WPB_P16 1
#endif
#ifndef DRL_STEP_WPB_P32
#define DRL_STEP_WPB_P32 1
#endif
constexpr int step_wpb(int P) { return P == 32 ? DRL_STEP_WPB_P32 : P == 16 ? DRL_STEP_WPB_P16 : 1; }
template <int P, class GEO, bool NT, bool CODE = false, bool RING = false>
__global__ void __launch_bounds__(64 * step_wpb(P))
__attribute__((amdgpu_waves_per_eu(P <= 8 ? 8 : (P == 32 ? DRL_STEP_WAVES_P32 : P == 16 ? DRL_STEP_WAVES_P16 : 1), 8)))
drl_step_kernel(StepArgs a) {
    constexpr int WPB = step_wpb(P);
    const int64_t batch = WPB == 1 ? (int64_t)xcd_block(blockIdx.x, gridDim.x)
                                   : (int64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    step_batch<P, GEO, false, NT, CODE, RING>(a, batch * (64 / P));
}

// drl_rollout: a.steps steps per launch, same wave layout (P >= 16).
template <int P, class GEO>
__global__ void __launch_bounds__(64) drl_rollout_kernel(StepArgs a) {
    step_batch<P, GEO, true, true>(a, (int64_t)xcd_block(blockIdx.x, gridDim.x) * (64 / P));
}

// ------------------------------------------------------------ observation ---
template <int P, class GEO>
__global__ void __launch_bounds__(64) drl_obs_kernel(StepArgs a) {
    constexpr int GPW = 64 / P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const GEO g{a};
    const int lane = threadIdx.x & 63;
    const int grp = lane / P;
    const int j = lane % P;
    const int64_t wenv0 = (int64_t)xcd_block(blockIdx.x, gridDim.x) * GPW;
    const int nenv_w = (int)min((int64_t)GPW, a.E - wenv0);
    if (nenv_w <= 0) return;
    const bool env_ok = grp < nenv_w;
    const int N = g.n();
    const WaveLds W = carve((l_u8*)smem, GPW, P, g);
    stage_ground_nib(a.ground + wenv0 * g.pstride(), nenv_w * g.pstride(), W.gl, lane, g.nib());
    lds_zero(W.paint, GPW * g.lds_paint(), lane);
    const bool active = env_ok && j < N;
    const uint32_t rec = active ? a.drones[wenv0 * N + (uint32_t)(grp * N + j)] : 0u;
    const int y = rec & 255u, x = (rec >> 8) & 255u;
    const int c = (rec >> 16) & 255u, carry = (rec >> 24) & 1u;
    const int idx = ((int)(rec >> 25) < N) ? (int)(rec >> 25) : j;
    l_u16* posidx = W.posidx + grp * g.np();
    if (active) posidx[idx] = (uint16_t)(y * g.side() + x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (active) paint_windows(W.paint + grp * g.lds_paint(), posidx, y, x, (uint8_t)((c + 1) | (carry << 7)), g);
    wave_sync();
    float* obase = a.obs + wenv0 * (int64_t)(6u * g.env_cells());
    uint16_t* crow = a.code ? code_row(a, wenv0, g) : nullptr;
    l_u16* cst = reinterpret_cast<l_u16*>((l_u8*)smem + a.code_lds);
    if (!a.code) write_obs_wave(obase, nenv_w, g, W, a.obs_wide, lane);
    else if (a.obs) write_obs_wave<false, true, true>(obase, nenv_w, g, W, a.obs_wide, lane, crow, cst);
    else write_obs_wave<false, true, false>(obase, nenv_w, g, W, a.obs_wide, lane, crow, cst);
}

// ------------------------------------------------------------------ reset ---
// One lane per env.  Per-lane LDS: shuffle list u16[cells] (+ pool copy for
// Random.sample's pool branch) and the selected-index list u16[64].
struct ResetLane {
    uint32_t* mrow;
    int midx;
};

// init_genrand(19650218), the constant start of every init_by_array.
struct MtInitTable {
    uint32_t v[MT_N];
    constexpr MtInitTable() : v() {
        v[0] = 19650218u;
        for (int i = 1; i < MT_N; i++) v[i] = 1812433253u * (v[i - 1] ^ (v[i - 1] >> 30)) + (uint32_t)i;
    }
};
__constant__ MtInitTable kMtInit = MtInitTable();

// random.seed(seed) for 0 <= seed < 2**64 (init_by_array with its 32-bit words).
__device__ void mt_seed_row(uint32_t* row, uint64_t seed) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const int keylen = k1 ? 2 : 1;
    int i = 1, jj = 0;
    uint32_t prev = kMtInit.v[0];
    uint32_t m1 = 0;  // value of mt[1] written by the first pass
    // first pass: MT_N iterations (keylen <= 2 < MT_N)
    for (int k = 0; k < MT_N; ++k) {
        const uint32_t base = (k < MT_N - 1) ? kMtInit.v[i] : m1;  // the last iteration revisits i = 1
        const uint32_t key = jj == 0 ? k0 : k1;
        const uint32_t v = (base ^ ((prev ^ (prev >> 30)) * 1664525u)) + key + (uint32_t)jj;
        row[i] = v;
        if (i == 1 && k == 0) m1 = v;
        prev = v;
        ++i;
        ++jj;
        if (i >= MT_N) {
            row[0] = row[MT_N - 1];
            prev = row[0];
            i = 1;
        }
        if (jj >= keylen) jj = 0;
    }
    // second pass: MT_N-1 iterations starting at i = 2
    for (int k = 0; k < MT_N - 1; ++k) {
        const uint32_t cur = row[i];
        const uint32_t v = (cur ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        row[i] = v;
        prev = v;
        ++i;
        if (i >= MT_N) {
            row[0] = row[MT_N - 1];
            prev = row[0];
            i = 1;
        }
    }
    row[0] = 0x80000000u;
}

// random.seed(seed) for a whole wave's register copy of the row (x[c] lane l
// = mt[64c + l], as twist_regs): the same init_by_array passes as mt_seed_row,
// run as a scalar chain -- each step reads its word with readlane, mixes it in
// SGPRs and writes it back into its lane (no memory round trips).
__device__ __forceinline__ void mt_seed_regs(uint32_t (&x)[10], uint64_t seed, int lane) {
#pragma unroll
    for (int c = 0; c < 10; ++c) x[c] = (64 * c + lane < MT_N) ? kMtInit.v[64 * c + lane] : 0u;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const uint32_t two = k1 ? 1u : 0u;  // key length 2: key words alternate, j = 0, 1, 0, ...
    uint32_t prev = kMtInit.v[0], jj = 0;
    auto rd = [](uint32_t v, int l) __attribute__((always_inline)) {
        return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
    };
    auto wr = [lane](uint32_t v, int l, uint32_t old) __attribute__((always_inline)) { return lane == l ? v : old; };
    // pass 1 (random.c init_by_array: k = max(N, keylen) steps): i = 1..623 ...
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int lend = c == 9 ? MT_N - 576 : 64;
        for (int l = c == 0 ? 1 : 0; l < lend; ++l) {
            const uint32_t v = (rd(x[c], l) ^ ((prev ^ (prev >> 30)) * 1664525u)) + (jj ? k1 + 1u : k0);
            x[c] = wr(v, l, x[c]);
            prev = v;
            jj ^= two;
        }
    }
    prev = rd(x[9], MT_N - 577);  // ... mt[0] = mt[623], then i = 1 once more
    x[0] = wr(prev, 0, x[0]);
    prev = (rd(x[0], 1) ^ ((prev ^ (prev >> 30)) * 1664525u)) + (jj ? k1 + 1u : k0);
    x[0] = wr(prev, 1, x[0]);
    // pass 2 (N - 1 steps): i = 2..623, mt[0] = mt[623], i = 1
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int lend = c == 9 ? MT_N - 576 : 64;
        for (int l = c == 0 ? 2 : 0; l < lend; ++l) {
            const uint32_t v = (rd(x[c], l) ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)(64 * c + l);
            x[c] = wr(v, l, x[c]);
            prev = v;
        }
    }
    prev = rd(x[9], MT_N - 577);
    x[0] = wr(prev, 0, x[0]);
    prev = (rd(x[0], 1) ^ ((prev ^ (prev >> 30)) * 1566083941u)) - 1u;
    x[0] = wr(prev, 1, x[0]);
    x[0] = wr(0x80000000u, 0, x[0]);  // mt[0] = 0x80000000
}

__global__ void __launch_bounds__(64) drl_reset_kernel(ResetArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int64_t env = (int64_t)blockIdx.x * a.lanes + lane;
    const bool own = lane < a.lanes && env < a.E && (a.mask == nullptr || a.mask[env] != 0);
    uint16_t* list = reinterpret_cast<uint16_t*>(smem + (size_t)lane * a.lane_lds);
    uint16_t* sel = list + a.list_cap;
    uint16_t* pool = sel + 64;
    const int GG = a.cells, N = a.n_drones;
    const uint32_t w0 = (own && !a.reseed) ? a.mt_index[env] : 0u;
    const int par = mi_par(w0);  // the block holding the stream (a reseed writes block 0)
    uint32_t* mrow = a.mt + (own ? env : 0) * MT_WORDS + par * MT_ALT;
    uint8_t* grow = a.ground + (own ? env : 0) * a.gstride;

    if (own) {
        if (a.reseed) mt_seed_row(mrow, a.seed_base + (uint64_t)env);
        for (int v = 0; v < a.gstride / 16; ++v) reinterpret_cast<uint4*>(grow)[v] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = 0; i < GG; ++i) list[i] = (uint16_t)i;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zeroed rows before the nibble ORs
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int midx = own ? (a.reseed ? MT_N : min(mi_idx(w0), MT_N)) : MT_N;
    int n = GG;

    // Draw one tempered output for every participating lane; twists are
    // cooperative over the whole wave.
#define DRL_DRAW_LOOP(PHASE_ACTIVE, ...)                                                  \
    for (;;) {                                                                            \
        const bool act_ = own && (PHASE_ACTIVE);                                          \
        if (!__ballot(act_)) break;                                                       \
        uint64_t need_ = __ballot(act_ && midx >= MT_N);                                  \
        while (need_) {                                                                   \
            const int tl_ = __ffsll((unsigned long long)need_) - 1;                       \
            need_ &= need_ - 1ull;                                                        \
            twist_wave(a.mt + ((int64_t)blockIdx.x * a.lanes + tl_) * MT_WORDS +             \
                           __builtin_amdgcn_readlane(par, tl_) * MT_ALT, lane);               \
            if (lane == tl_) midx = 0;                                                    \
        }                                                                                 \
        if (act_) {                                                                       \
            const uint32_t u = temper(load_l2(mrow + midx));                              \
            ++midx;                                                                       \
            __VA_ARGS__                                                                   \
        }                                                                                 \
    }

    // Random.shuffle(list[0:n]) (random.py:380-395)
#define DRL_SHUFFLE(NLEN)                                                    \
    {                                                                       \
        int si = (NLEN) - 1;                                                \
        DRL_DRAW_LOOP(si >= 1, {                                            \
            const uint32_t rr = u >> (32 - bitlen((uint32_t)si + 1u));      \
            if ((int)rr <= si) {                                            \
                const uint16_t t = list[si];                                \
                list[si] = list[rr];                                        \
                list[rr] = t;                                               \
                --si;                                                       \
            }                                                               \
        })                                                                  \
    }

    // skyscrapers: shuffle, pop from the end (env.py:58-66,83-84)
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_sky; ++t) nib_or(grow, list[n - 1 - t], OBJ_SKYSCRAPER);
    n -= a.n_sky;

    // drones: Random.sample(list[0:n], N) (random.py:480-504, env.py:88-89)
    if (a.pool_branch) {
        if (own)
            for (int i = 0; i < n; ++i) pool[i] = list[i];
        int si = 0;
        DRL_DRAW_LOOP(si < N, {
            const uint32_t m = (uint32_t)(n - si);
            const uint32_t rr = u >> (32 - bitlen(m));
            if (rr < m) {
                sel[si] = pool[rr];
                pool[rr] = pool[m - 1u];
                ++si;
            }
        })
    } else {
        int si = 0;
        const int kb = bitlen((uint32_t)n);
        DRL_DRAW_LOOP(si < N, {
            const uint32_t rr = u >> (32 - kb);
            if ((int)rr < n) {
                bool seen = false;
                for (int q = 0; q < si; ++q) seen |= (sel[q] == rr);
                if (!seen) sel[si++] = (uint16_t)rr;
            }
        })
        if (own)
            for (int i = 0; i < N; ++i) sel[i] = list[sel[i]];
    }

    // packets, dropzones, stations (env.py:91-96)
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_pack; ++t) nib_or(grow, list[n - 1 - t], OBJ_PACKET);
    n -= a.n_pack;
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_drop; ++t) nib_or(grow, list[n - 1 - t], OBJ_DROPZONE);
    n -= a.n_drop;
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_stat; ++t) nib_or(grow, list[n - 1 - t], OBJ_STATION);
    n -= a.n_stat;
#undef DRL_SHUFFLE
#undef DRL_DRAW_LOOP

    // drones in index order (dict order 0..N-1), then _pick_packets_after_respawn
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the placements' nibble ORs have landed
    if (own) {
        for (int d = 0; d < N; ++d) {
            const int cell = sel[d];
            int carry = 0;
            if (nib_get_l2(grow, cell) == OBJ_PACKET) {
                carry = 1;
                nib_clear(grow, cell);
            }
            const uint32_t py = fdiv((uint32_t)cell, a.div_side);
            a.drones[env * N + d] = pack_drone((int)py, cell - (int)py * a.side, 100, carry, d);
        }
        a.mt_index[env] = mi_pack(midx, par, 0, 0);  // the candidate ring is stale: empty
    }
}

// ------------------------------------------------------- reset (wave/env) ---
__device__ __forceinline__ int mbcnt64(uint64_t m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Up to 64 consecutive Fisher-Yates steps of Random.shuffle (random.py:380-395)
// at once: lane l holds the stream's draw 64c + l (u, tempered), lanes
// [l0, l1) are unconsumed.  Returns the first lane NOT consumed; si and the
// list advance exactly as the one-draw-at-a-time loop would leave them.
//  1. acceptance: draw k is consumed iff fewer than si0 draws before it were
//     accepted, and accepted iff r_k = u_k >> (32 - bitlen(s_k + 1)) <= s_k
//     with s_k = si0 - (#accepted before k).  When bitlen(s + 1) is the same
//     for every s the chunk can reach (all but ~12 chunks of a shuffle), r_k is
//     fixed and #accepted-before lies in [0, k - l0]: one ballot of each bound
//     decides every lane outside a narrow band; lanes inside it (and chunks
//     whose width changes) iterate the ballot to its fixed point, lanes
//     settling left to right.
//  2. accepted draw t (rank t among them) swaps i_t = si0 - t with j_t = r_t.
//     With A_t / B_t the values at i_t / j_t just before step t: i_t ends as
//     B_t (later steps only touch smaller positions); A_t = A_p, p = the last
//     earlier step whose j was i_t (else the original list[i_t]); B_t = A_q,
//     q = the last earlier step with the same j (else the original list[j_t]);
//     each j position ends as A of its last writer.
//     * p: the lanes whose j lies in the chunk's own i range are found by a
//       compare (no LDS); an ascending readlane pass hands each one's A to
//       the lane owning that i (ascending = the last writer wins, and its own
//       A is final by then).  About 1.3 such lanes per chunk on average at
//       64x64; past `serial_chains` of them (small lists, the ends of
//       shuffles) a 64-slot table keeps the last writer per i slot and the
//       chains are pointer-jumped with bpermutes instead.
//     * q: a bitmap of j's (one bit per cell) OR-ed with return in the same
//       LDS round trip as the list reads: a lane that finds its bit set has
//       a repeated j (which lane of a pair sees it does not matter); each
//       repeated-j group is then ordered by lane with readlanes.
//     The bitmap bits are cleared by an AND after the writes.
__device__ __forceinline__ uint64_t bal(bool b) { return __builtin_amdgcn_ballot_w64(b); }

struct FyLds {  // the batched shuffle's LDS: list (+ dummy slots at list index `dummy`), j bitmap, i-slot table
    uint16_t* list;
    uint32_t* bmap;
    uint32_t* ptab;
    int dummy;
    int bmask, bshift;  // cell j -> bitmap word j & bmask, bit j >> bshift (>= 64 words: few lanes per word)
    int serial_chains;
};

__device__ __forceinline__ void fy_swaps(const FyLds& f, uint64_t S, int m, bool acc, int t, uint32_t r, int si0,
                                         int lane) {
    uint16_t* const list = f.list;
    uint32_t* const ptab = f.ptab;
    const int j = acc ? (int)r : 0;
    const int ii = si0 - t;    // >= 0 on every lane (t <= m <= si0)
    const int slot = si0 - j;  // j's rank if j lies in the i range; rejected lanes: si0 >= m, none
    const uint32_t bit = acc ? 1u << (j >> f.bshift) : 0u;
    // (rejected lanes OR / AND a zero bit into a word of their own: with one
    // shared word (j = 0) their ~18 atomics per chunk serialised on one bank,
    // C5 17.6e6 -> 19.3e6 resets/s; zeroing the whole bitmap with plain
    // stores instead of the AND measured slower, 18.1e6, and so did skipping
    // the rejected lanes' atomics under an exec mask, 18.9e6, while a dword
    // per dummy slot changed nothing; profiles/r03_reset_occ/)
    uint32_t* const pw = f.bmap + ((acc ? j : lane) & f.bmask);
    uint16_t* const pi = list + ii;
    uint16_t* const pj = list + j;
    uint16_t* const pd = list + f.dummy + lane;
    const uint32_t a0 = *pi;
    const uint32_t l0j = *pj;
    const uint32_t old = __hip_atomic_fetch_or(pw, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    uint64_t W = bal(slot < m);  // writers into the i range (self-swaps included: a no-op below)
    uint32_t A = a0;
    if (W == 0) {
        // no lane writes into the chunk's own i range (most chunks of a large list)
    } else if (popc(W) <= f.serial_chains) {
        do {  // ascending: the lane owning i = j takes this lane's A (rejected lanes' A is never stored)
            const int k = lobit(W);
            W &= W - 1;
            const int sk = __builtin_amdgcn_readlane(slot, k);
            const uint32_t ak = (uint32_t)__builtin_amdgcn_readlane((int)A, k);
            if (t == sk) A = ak;
        } while (W);
    } else {  // many (small lists): last writer per i slot, then pointer jumping to the chain roots
        const bool w = slot < m && slot != t;
        if (w) __hip_atomic_fetch_max(ptab + slot, (uint32_t)lane + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        wave_sync();
        const uint32_t pv = acc ? ptab[t] : 0u;
        wave_sync();
        if (w) ptab[slot] = 0u;
        int f = pv ? (int)pv - 1 : lane;
        for (;;) {
            const int f2 = __shfl(f, f);
            if (!bal(f2 != f)) break;
            f = f2;
        }
        A = __shfl(a0, f);
    }
    uint64_t D = bal((old & bit) != 0u);
    uint32_t B = l0j;
    bool jw = acc;  // this lane writes its j position (the last writer of each repeated j does)
    if (D) {
        uint64_t notlast = 0;
        do {  // one repeated-j group per pass; B of each member = A of the member below it
            const int jk = __builtin_amdgcn_readlane(j, lobit(D));
            uint64_t G = bal(j == jk) & S;
            D &= ~G;
            const int lo = lobit(G), hi = hibit(G);
            notlast |= G & ~(1ull << hi);
            if (popc(G) == 2) {  // a pair (nearly always): one readlane
                const uint32_t ab = (uint32_t)__builtin_amdgcn_readlane((int)A, lo);
                if (lane == hi) B = ab;
            } else {
                int below = lo;
                G &= G - 1;
                while (G) {
                    const int x = lobit(G);
                    G &= G - 1;
                    const uint32_t ab = (uint32_t)__builtin_amdgcn_readlane((int)A, below);
                    if (lane == x) B = ab;
                    below = x;
                }
            }
        } while (D);
        jw = acc && !((notlast >> lane) & 1ull);
    }
    // j positions first (i-range ones are rewritten next), then the i positions
    *(jw ? pj : pd) = (uint16_t)A;
    *(acc ? pi : pd) = (uint16_t)B;
    __hip_atomic_fetch_and(pw, ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    wave_sync();
}

// A chunk anywhere in a shuffle (its first draws, the shuffle's end, a
// count-only chunk): returns the first lane NOT consumed.
__device__ __forceinline__ int fy_chunk(const FyLds& f, uint32_t u, int lane, uint64_t lanebit, int l0, int l1, int& si,
                                        bool count_only) {
    const int si0 = si;
    const bool valid = lane >= l0 && lane < l1;
    const int kb = bitlen((uint32_t)si0 + 1u);
    const int slo = si0 - (l1 - 1 - l0);  // the smallest s a draw of this chunk can see
    const bool uniform = slo >= 1 && bitlen((uint32_t)slo + 1u) == kb;
    uint64_t S;
    uint32_t r = u >> (32 - kb);
    if (uniform) {
        const uint64_t H = bal(valid & ((int)r <= si0));
        S = H;
        if (bal(valid & ((int)r + (lane - l0) <= si0)) != H) {
            for (;;) {
                const uint64_t S2 = bal(valid & ((int)r + mbcnt64(S) <= si0));
                if (S2 == S) break;
                S = S2;
            }
        }
    } else {
        S = bal(valid);
        for (;;) {
            const int sk = si0 - mbcnt64(S);
            const uint32_t rk = u >> (32 - bitlen((uint32_t)max(sk, 1) + 1u));
            const uint64_t S2 = bal(valid & (sk >= 1) & ((int)rk <= sk));
            if (S2 == S) break;
            S = S2;
        }
        r = u >> (32 - bitlen((uint32_t)max(si0 - mbcnt64(S), 1) + 1u));
    }
    const int m = popc(S);
    si = si0 - m;
    const int consumed = si == 0 ? hibit(S) + 1 : l1;
    if (m != 0 && !count_only) fy_swaps(f, S, m, (S & lanebit) != 0ull, mbcnt64(S), r, si0, lane);
    return consumed;
}

// The reset's hot loop: whole chunks of one shuffle while every draw of a
// chunk sees s >= 1 (the shuffle cannot end inside it), the register twist
// inline, no phase bookkeeping.  Enters at a chunk boundary (midx % 64 == 0,
// or MT_N: twist first); the chunk's register x[c] is read with a uniform
// register index.  Chunks that start below swap_floor only count (the
// stations' shuffle needs its top positions only).  Returns with midx at the
// first chunk that could end the shuffle (the caller's general path takes it).
__device__ __forceinline__ void fy_run(const FyLds& f, uint32_t (&x)[10], int& midx, int& si, int swap_floor, int lane) {
    int c = midx >> 6;
    if (midx >= MT_N) {
        twist_regs(x, lane);
        c = 0;
    }
    int cnt = c == 9 ? MT_N - 576 : 64;
    // Acceptance as one fixed-point loop for every chunk (the scalar unit is
    // the reset's bottleneck, the vector units are not): start from "every
    // draw below was accepted" (s_k = si0 - k, the smallest s each can see)
    // and re-evaluate with the ranks that gives, until the set repeats.  With
    // one draw width over the chunk and no draw in the narrow band, the start
    // is already exact and the loop runs twice.
    while (si - cnt >= 1) {
        const int si0 = si;
        const uint32_t u = temper(x[__builtin_amdgcn_readfirstlane(c)]);
        const bool live = lane < cnt;  // chunk 9 holds 48 words
        const uint64_t L = bal(live);
        auto accept = [&](int tk) __attribute__((always_inline)) {  // tk: accepted draws below this lane
            const int sk = si0 - tk;  // >= 1 on every live lane
            return bal((int)(u >> __builtin_clz((uint32_t)sk + 1u)) <= sk) & L;
        };
        int t = lane;  // the start: every draw below accepted (= mbcnt of all lanes)
        uint64_t S = accept(t), Sp = ~0ull;
        while (S != Sp) {
            Sp = S;
            t = mbcnt64(S);
            S = accept(t);
        }
        const uint32_t r = u >> __builtin_clz((uint32_t)(si0 - t) + 1u);
        const bool acc = live & ((int)r <= si0 - t);
        const int m = popc(S);
        if (si0 >= swap_floor) fy_swaps(f, S, m, acc, t, r, si0, lane);
        si = si0 - m;
        if (++c == 10) {
            twist_regs(x, lane);
            c = 0;
        }
        cnt = c == 9 ? MT_N - 576 : 64;
    }
    midx = 64 * c;
}

// One wavefront per env, for large grids (the lane-per-env kernel above is
// LDS-bound to a few envs per CU there, and each of its ~22k serial draws at
// 64x64 is a memory round trip).  The env's MT state stays in registers
// (lane l holds words 64c + l) and twists in registers; a draw is a readlane
// of the current tempered 64-word chunk, so the shuffle chain is uniform
// scalar control flow plus single-lane LDS swaps.  Same draws, same order,
// same results as the lane kernel (and the reference).
// WPB waves per workgroup, each its own env and LDS image (no workgroup barrier): a CU runs at most 16
// workgroups, so one-wave workgroups cap it at 16 resets in flight where the LDS would hold more (small grids).
template <int WPB>
__global__ void __launch_bounds__(64 * WPB) drl_reset_wave_kernel(ResetArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
    const int lane = threadIdx.x & 63;
    const int wv = WPB > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    unsigned char* const smem = smem_all + (size_t)wv * a.wave_lds;
    const int64_t env = (int64_t)blockIdx.x * WPB + wv;
    if (env >= a.E || (a.mask != nullptr && a.mask[env] == 0)) return;  // whole wave, uniform
    FyLds f;
    f.bmap = reinterpret_cast<uint32_t*>(smem);  // batched shuffle: one bit per cell (repeated j's)
    f.bmask = a.fy_bwords - 1;
    f.bshift = __builtin_ctz((unsigned)a.fy_bwords);
    f.ptab = f.bmap + a.fy_bwords;  // ... and the last writer per i slot (many chains)
    f.list = reinterpret_cast<uint16_t*>(f.ptab + 64);
    f.dummy = a.list_cap + 64;  // 64 u16 slots the batched shuffle's rejected lanes store into
    f.serial_chains = a.fy_serial;
    uint32_t* const bmap = f.bmap;
    uint16_t* list = f.list;
    uint16_t* sel = list + a.list_cap;
    uint16_t* pool = sel + 128;
    const uint64_t lanebit = 1ull << lane;
    const int GG = a.cells, N = a.n_drones;
    const uint32_t w0 = a.reseed ? 0u : a.mt_index[env];
    const int par = mi_par(w0);  // the block holding the stream (a reseed writes block 0)
    uint32_t* mrow = a.mt + env * MT_WORDS + par * MT_ALT;
    uint8_t* grow = a.ground + env * a.gstride;
    for (int i = lane; i < a.fy_bwords + 64; i += 64) bmap[i] = 0u;

    // x[c] holds words 64c + lane; the current chunk's register is read with
    // a uniform register index (s_set_gpr_idx), no data movement
    int midx = a.reseed ? MT_N : min(mi_idx(w0), MT_N);
    int rot = midx < MT_N ? midx >> 6 : 0;
    uint32_t x[10];
    if (a.reseed) {
        mt_seed_regs(x, a.seed_base + (uint64_t)env, lane);
    } else {
#pragma unroll
        for (int c = 0; c < 10; ++c) x[c] = (64 * c + lane < MT_N) ? load_l2(mrow + 64 * c + lane) : 0u;
    }
    for (int v = lane; v < a.gstride / 16; v += 64) reinterpret_cast<uint4*>(grow)[v] = make_uint4(0u, 0u, 0u, 0u);
    for (int i = lane; i < GG; i += 64) list[i] = (uint16_t)i;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zeroed row before the nibble ORs
    uint32_t tcur = temper(x[__builtin_amdgcn_readfirstlane(rot)]);
    wave_sync();

    // The reset as a phase machine with ONE draw site (the register twist is
    // inlined once): 0 shuffle for the skyscrapers, 1 sample the drones, 2-4
    // shuffles for packets / dropzones / stations (env.py:68-101, random.py
    // shuffle :380-395 and sample :480-504).
    const int kb = bitlen((uint32_t)(GG - a.n_sky));  // sample's set branch: randbelow(n) bits
    int n = GG, phase = 0, si = GG - 1;
    uint32_t mine = 0xffffffffu;  // set branch: lane q < N holds selection q
    auto place = [&](int count, uint8_t code) __attribute__((always_inline)) {  // pop `count` from the end
        wave_sync();
        for (int t = lane; t < count; t += 64) nib_or(grow, list[n - 1 - t], code);  // (packed row: atomic ORs)
        n -= count;
    };
    // finish phases that need no (more) draws; set up the next one
    auto settle = [&]() __attribute__((always_inline)) {
        for (;;) {
            if (phase == 0 && si < 1) {
                place(a.n_sky, OBJ_SKYSCRAPER);
                phase = 1;
                si = 0;
                if (a.pool_branch) {
                    for (int i = lane; i < n; i += 64) pool[i] = list[i];
                    wave_sync();
                }
            } else if (phase == 1 && si >= N) {
                if (!a.pool_branch && lane < N) sel[lane] = list[mine];
                wave_sync();
                phase = 2;
                si = n - 1;
            } else if (phase >= 2 && phase <= 4 && si < 1) {
                place(phase == 2 ? a.n_pack : phase == 3 ? a.n_drop : a.n_stat,
                      phase == 2 ? OBJ_PACKET : phase == 3 ? OBJ_DROPZONE : OBJ_STATION);
                ++phase;
                si = n - 1;
            } else {
                return;
            }
        }
    };
    DRL_RS_DECL;
    DRL_SUBT(rs_tt);
    settle();
    while (phase <= 4) {
        // ---- the current 64-word chunk of the env's stream (twist first when
        // it is used up): the single twist site
        DRL_RS_BEGIN();
        if (midx >= MT_N) {
            twist_regs(x, lane);
            midx = 0;
            rot = 0;
            tcur = temper(x[0]);
            DRL_RS_COUNT(7);
        } else if ((midx >> 6) != rot) {  // next chunk
            rot = midx >> 6;
            tcur = temper(x[__builtin_amdgcn_readfirstlane(rot)]);
        }
        DRL_RS_END(1);
        const int c = rot;
        const int end = min(64 * c + 64, MT_N);
        // ---- consume the chunk's draws for the current phase (tight loops;
        // si / midx stay uniform; readlane returns int: shift it as uint32)
        if (phase != 1 && si > 64 && (midx & 63) == 0 && a.fy_batch_min <= 1) {
            // the hot loop from a chunk boundary until the shuffle's last chunk
            fy_run(f, x, midx, si, phase == 4 ? n - a.n_stat : 0, lane);
            rot = -1;  // x may have twisted: re-select the chunk
            continue;
        } else if (phase != 1 && si >= a.fy_batch_min) {
            // the last shuffle only needs its top n_stat positions: below them
            // the draws are consumed without swapping
            const bool count_only = phase == 4 && si < n - a.n_stat;
            DRL_RS_BEGIN();
            midx = 64 * c + fy_chunk(f, tcur, lane, lanebit, midx - 64 * c, end - 64 * c, si, count_only);
            DRL_RS_END(count_only ? 2 : 0);
            DRL_RS_COUNT(count_only ? 8 : 6);
            if (si != 0) continue;  // the shuffle goes on: nothing to settle
        } else if (phase != 1) {  // Fisher-Yates steps of a shuffle, one draw at a time; lane 0 swaps
            DRL_RS_BEGIN();
            int kb_s = bitlen((uint32_t)si + 1u);
            while (midx < end && si >= 1) {
                const uint32_t rr = (uint32_t)__builtin_amdgcn_readlane(tcur, midx & 63) >> (32 - kb_s);
                ++midx;
                if ((int)rr <= si) {
                    const uint16_t vi = list[si], vr = list[rr];  // broadcast reads
                    if (lane == 0) {
                        list[si] = vr;
                        list[rr] = vi;
                    }
                    --si;
                    kb_s = bitlen((uint32_t)si + 1u);
                }
            }
            DRL_RS_END(3);
        } else if (a.pool_branch) {
            while (midx < end && si < N) {
                const uint32_t m = (uint32_t)(n - si);
                const uint32_t rr = (uint32_t)__builtin_amdgcn_readlane(tcur, midx & 63) >> (32 - bitlen(m));
                ++midx;
                if (rr < m) {
                    const uint16_t pr = pool[rr], pl = pool[m - 1u];
                    if (lane == 0) {
                        sel[si] = pr;
                        pool[rr] = pl;
                    }
                    ++si;
                }
            }
        } else {
            DRL_RS_BEGIN();
            while (midx < end && si < N) {
                const uint32_t rr = (uint32_t)__builtin_amdgcn_readlane(tcur, midx & 63) >> (32 - kb);
                ++midx;
                if ((int)rr < n && !__ballot(lane < si && mine == rr)) {
                    if (lane == si) mine = rr;
                    ++si;
                }
            }
            DRL_RS_END(4);
        }
        DRL_RS_BEGIN();
        settle();
        DRL_RS_END(5);
    }
    wave_sync();
#ifdef DRL_STAMPS
    DRL_SUBT(rs_t1);
    rs_acc[9] = rs_t1 - rs_tt;
    if (lane == 0 && g_stamps)
        for (int k = 0; k < 10; ++k) g_stamps[env * 16 + k] = rs_acc[k];
#endif

    // drones in index order (dict order 0..N-1), then _pick_packets_after_respawn
    // (distinct cells: parallel)
    if (lane < N) {
        const int cell = sel[lane];
        int carry = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the placements' ORs have landed
        if (nib_get_l2(grow, cell) == OBJ_PACKET) {
            carry = 1;
            nib_clear(grow, cell);
        }
        const uint32_t py = fdiv((uint32_t)cell, a.div_side);
        a.drones[env * N + lane] = pack_drone((int)py, cell - (int)py * a.side, 100, carry, lane);
    }
#pragma unroll
    for (int c = 0; c < 10; ++c)
        if (64 * c + lane < MT_N) mrow[64 * c + lane] = x[c];
    if (lane == 0) a.mt_index[env] = mi_pack(midx, par, 0, 0);  // the candidate ring is stale: empty
}

// ------------------------------------------------------------ full grid ---
// GridView observation (wrappers.py:10-31,34-43): the [side][side][6] base grid
// of every env, the same grid every drone of the env sees.  One 256-thread
// block per env: drones paint their air byte ((charge+1) | carry<<7) into an
// LDS image of the cells, then every cell is written as 6 floats (three 8-B
// stores).  ch4 = charge/100 exactly as the windowed observation computes it.
__global__ void __launch_bounds__(256) drl_grid_obs_kernel(const uint8_t* __restrict__ ground,
                                                           const uint32_t* __restrict__ drones, int side, int N,
                                                           int gstride, float* __restrict__ out) {
    extern __shared__ uint8_t air[];
    const int64_t e = blockIdx.x;
    const int cells = side * side;
    for (int c = threadIdx.x; c < cells; c += blockDim.x) air[c] = 0;
    __syncthreads();
    if ((int)threadIdx.x < N) {
        const uint32_t r = drones[e * N + threadIdx.x];
        const int y = r & 255u, x = (r >> 8) & 255u;
        if (y < side && x < side) air[y * side + x] = (uint8_t)((((r >> 16) & 255u) + 1) | (((r >> 24) & 1u) << 7));
    }
    __syncthreads();
    const uint8_t* g = ground + e * gstride;
    float2* o = reinterpret_cast<float2*>(out + e * (int64_t)cells * 6);
    for (int c = threadIdx.x; c < cells; c += blockDim.x) {
        const uint32_t obj = nib_get(g, c), a = air[c];
        o[3 * c] = make_float2(a ? 1.0f : 0.0f, (obj == OBJ_PACKET || (a & 0x80u)) ? 1.0f : 0.0f);
        o[3 * c + 1] = make_float2(obj == OBJ_DROPZONE ? 1.0f : 0.0f, obj == OBJ_STATION ? 1.0f : 0.0f);
        o[3 * c + 2] = make_float2(a ? div100((int)(a & 0x7fu) - 1) : 0.0f, obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f);
    }
}

// ------------------------------------------------------- decode / encode ---
__global__ void drl_decode_kernel(const uint32_t* __restrict__ drones, int64_t total, int N, int32_t* order,
                                  int32_t* yv, int32_t* xv, int32_t* cv, uint8_t* kv) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t e = t / N;
    const uint32_t r = drones[t];
    const int idx = r >> 25;
    const int64_t o = e * N + idx;
    if (order) order[t] = idx;
    if (yv) yv[o] = r & 255u;
    if (xv) xv[o] = (r >> 8) & 255u;
    if (cv) cv[o] = (r >> 16) & 255u;
    if (kv) kv[o] = (r >> 24) & 1u;
}

__global__ void drl_encode_kernel(uint32_t* __restrict__ drones, int64_t total, int N, const int32_t* order,
                                  const int32_t* yv, const int32_t* xv, const int32_t* cv, const uint8_t* kv) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int64_t e = t / N;
    const int idx = order[t];
    const int64_t o = e * N + idx;
    drones[t] = pack_drone(yv[o], xv[o], cv[o], kv[o] ? 1 : 0, idx);
}

// random.getstate() / setstate() words of every env: [E][625] = the 624
// words of the block holding the stream + the index.  CPython's setstate
// rejects an index outside [0, 624]; the kernels' MT reads assume that range,
// so set clamps and flags instead.  set writes block 0 and an empty ring.
__global__ void drl_mt_get_kernel(const uint32_t* __restrict__ mt, const uint32_t* __restrict__ mt_index, int64_t E,
                                  uint32_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= E * 625) return;
    const int64_t e = t / 625;
    const int k = (int)(t - e * 625);
    const uint32_t w = mt_index[e];
    out[t] = k < MT_N ? mt[e * MT_WORDS + mi_par(w) * MT_ALT + k] : (uint32_t)min(mi_idx(w), MT_N);
}

__global__ void drl_mt_set_kernel(uint32_t* __restrict__ mt, uint32_t* __restrict__ mt_index, int64_t E,
                                  const uint32_t* __restrict__ in, int32_t* err) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= E * 625) return;
    const int64_t e = t / 625;
    const int k = (int)(t - e * 625);
    if (k < MT_N) {
        mt[e * MT_WORDS + k] = in[t];
    } else {
        uint32_t idx = in[t];
        if (idx > (uint32_t)MT_N) {
            idx = (uint32_t)MT_N;
            if (err) atomicOr(err, DRL_ERR_BAD_STATE);
        }
        mt_index[e] = mi_pack((int)idx, 0, 0, 0);
    }
}

// ---------------------------------------------------------------- refill ---
// drl_refill: extend each env's respawn-candidate ring (include/dronerl.h)
// through the end of the MT block after the stream's, converting that block
// while its words are in registers.  The candidates are the (y, x) pairs of
// consecutive accepted randint(0, side-1) draws (_randbelow: the top kbits
// bits of a tempered word, kept if < side; env.py:226-233 draws y then x), in
// stream order from the end of the ring's last entry (or from the stream
// position when it is empty).  They depend on the stream alone, so they can be
// drawn ahead of the steps that consume them.
//
// An env needs a conversion when its ring does not reach past the stream's
// block s (after a reset or drl_mt_set, and once its stream has moved on into
// block s+1, whose entries the ring then still holds).  The conversion loads
// block s (2.5 KB, one round trip), converts its words from the ring's end on,
// twists it into block s+1 in registers, stores s+1 to the other block's words
// (the stream's own block is never written: get_state and every kernel that
// draws from the stream directly see the state its index says), and converts
// all of s+1.  Every MT word is thus read once, twisted once and written once
// (~9 B per word with its entry), instead of being re-read by 64-word passes
// after the twist that wrote it (round 2's refill: ~13 B per word).
//
// A wave serves kRefillEnvs envs (its 624 words each in x[e][10] as in
// twist_regs), four waves per workgroup: the mt_index and ring-end words of
// all of them are read at once, then the blocks of those that need a
// conversion, then they are converted one after another.  One env per wave
// measured best (C3 48.8 / 52.9 / 62.9 / 74.2 us per refill at 1 / 2 / 4 / 8
// envs per wave with chained chunks, tools/refill_time.py): a conversion is a
// latency chain, and more waves hide it better than shared round trips do.
// Within a 64-word chunk acceptance is one ballot, a draw's accepted rank an
// mbcnt, and an x draw takes its y from the previous accepted lane by
// ds_bpermute (the first of a chunk from the pending y carried from the
// previous chunk).  (Three passes that made the ten chunks of a block
// independent -- every ballot, then the pairing state in scalar registers,
// then the pairs -- measured slower: C3 60 vs 48 us, C5 134 vs 102.)  A ring
// that would overflow stops at DRL_CAND_SLOTS entries; its end then lies
// inside block s+1, whose words the next conversion (after the stream moves
// into s+1) converts from registers.
#ifndef DRL_REFILL_ENVS
#define DRL_REFILL_ENVS 1
#endif
constexpr int kRefillEnvs = DRL_REFILL_ENVS;  // envs per wave
constexpr int kRefillWaves = 4;               // waves per workgroup

// The conversion of one env whose stream block is in x (see above).
__device__ __forceinline__ void refill_env(const RefillArgs& a, int64_t env, uint32_t mw, uint32_t rend, int from,
                                           uint32_t (&x)[10], int lane) {
    uint32_t* const row = a.mt + env * MT_WORDS;
    const int cnt = mi_cnt(mw), spar = mi_par(mw);
    const int G = a.side, shift = 32 - a.kbits;
    const int room = CAND_Q - cnt;
    const int ring0 = mi_head(mw) + cnt;  // slot of the first new entry (mod CAND_Q)
    uint32_t* const ring = row + MT_RING;
    const uint64_t lower = (1ull << lane) - 1ull;
    int made = 0;             // entries written (uniform)
    int carry = 0, yv = 0;    // a pending y (accepted draw without its x yet)
    uint32_t end_word = rend; // ring-end word: MT index | block << 10 after the last entry
    // convert chunk c of block bp (positions >= f0 only)
    auto chunk = [&](uint32_t word, int c, int bp, int f0) __attribute__((always_inline)) {
        const int pos = 64 * c + lane;
        const bool valid = pos >= f0 && pos < MT_N;
        const int r = (int)(temper(word) >> shift);
        const bool acc = valid && r < G;
        const uint64_t M = __ballot(acc);
        const int k = mbcnt64(M);  // accepted draws of this chunk below this lane
        const int ar = carry + k;  // accepted rank within the pairing
        const uint64_t below = M & lower;
        const int yl = below ? 63 - __clzll((long long)below) : lane;
        const int ry = __shfl(r, yl);
        const int yy = k > 0 ? ry : yv;
        const int slot = made + (ar >> 1);
        const bool put = acc && (ar & 1) && slot < room;
        if (put) ring[(uint32_t)(ring0 + slot) & (uint32_t)(CAND_Q - 1)] = ce_pack(yy * G + r, pos + 1, bp);
        const uint64_t P = __ballot(put);
        if (P) end_word = (uint32_t)(64 * c + (63 - __clzll((long long)P)) + 1) | ((uint32_t)bp << 10);
        const int tot = carry + __popcll(M);
        if (M && (tot & 1)) yv = __builtin_amdgcn_readlane(r, 63 - __clzll((long long)M));
        made = min(made + (tot >> 1), room);
        carry = tot & 1;
    };
    // ---- the rest of the stream's block, from `from`
#pragma unroll
    for (int c = 0; c < 10; ++c)
        if (64 * c + 64 > from && made < room) chunk(x[c], c, spar, from);
    // ---- block s+1: twisted in registers, stored to the other block, converted
    twist_regs(x, lane);
    {
        uint32_t* dst = row + (uint32_t)(1 - spar) * MT_ALT;
#pragma unroll
        for (int c = 0; c < 10; ++c)
            if (64 * c + lane < MT_N) dst[64 * c + lane] = x[c];
    }
#pragma unroll
    for (int c = 0; c < 10; ++c)
        if (made < room) chunk(x[c], c, 1 - spar, 0);
    // (a pending y at the end is dropped: the next conversion re-reads it)
    if (lane == 0) {
        a.mt_index[env] = mi_pack(mi_idx(mw), spar, mi_head(mw), cnt + made);
        row[MT_RING_END] = end_word;
    }
}

__global__ void __launch_bounds__(64 * kRefillWaves) drl_refill_kernel(RefillArgs a) {
    constexpr int NE = kRefillEnvs;
    const int lane = threadIdx.x & 63;
    const int64_t env0 =
        ((int64_t)xcd_block(blockIdx.x, gridDim.x) * kRefillWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * NE;
    if (env0 >= a.E) return;  // whole wave
    // ---- round trip 1: each env's mt_index word and ring-end word (uniform: scalar loads)
    uint32_t mw[NE], rend[NE];
    int from[NE];
    bool need[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int64_t ev = min(env0 + e, a.E - 1);
        mw[e] = a.mt_index[ev];
        rend[e] = a.mt[ev * MT_WORDS + MT_RING_END];
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        // where the unconverted stream starts, relative to the stream's block:
        // the end of the ring's last entry (in the next block: + 624), or the
        // stream position when the ring is empty; nothing to do once the ring
        // reaches into the next block
        const int cnt = mi_cnt(mw[e]), spar = mi_par(mw[e]);
        from[e] = cnt > 0 ? min((int)(rend[e] & 0x3ffu), MT_N) + ((int)((rend[e] >> 10) & 1u) != spar ? MT_N : 0)
                          : min(mi_idx(mw[e]), MT_N);
        need[e] = env0 + e < a.E && from[e] <= MT_N;
    }
    // ---- round trip 2: the stream blocks of every env that needs a conversion
    // (not written by this kernel: plain loads), all issued before any is used
    uint32_t x[NE][10];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        if (need[e]) {
            const uint32_t* src = a.mt + (env0 + e) * MT_WORDS + (uint32_t)mi_par(mw[e]) * MT_ALT;
#pragma unroll
            for (int c = 0; c < 10; ++c) x[e][c] = (64 * c + lane < MT_N) ? src[64 * c + lane] : 0u;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < NE; ++e)
        if (need[e]) refill_env(a, env0 + e, mw[e], rend[e], from[e], x[e], lane);
}

// Worklist form (the default; DRL_REFILL_LIST=0 selects the wave-per-env
// kernel above): a workgroup owns kRefillListEnvs consecutive envs.  Its first
// wave reads their mt_index and ring-end words (one lane per env: two vector
// loads instead of a wave and two scalar round trips per env) and lists the
// envs that need a conversion in LDS; then the workgroup's waves take the
// listed envs in turn, so no wave is spent on an env with nothing to convert.
// At the benchmark cadences 40-60 % of the envs convert per refill, and a
// conversion moves ~5.6 KB (block s read, block s+1 written, ~156 entries):
// both forms run those bytes at ~5.6 TB/s, so the worklist saves only the
// per-env overhead: 2-6 % per refill, paired on identical states (C3 46.9 vs
// 50.0 us, C4 52.1 vs 52.3, C5 103.8 vs 106.3; 64 envs with 8 or 16 waves per
// workgroup measured no better; profiles/r03_refill/).
constexpr int kRefillListEnvs = 32, kRefillListWaves = 8;
template <int NENV, int NW>  // envs per workgroup (<= 64), waves per workgroup
__global__ void __launch_bounds__(64 * NW) drl_refill_list_kernel(RefillArgs a) {
    __shared__ uint32_t q_mw[64], q_rend[64];
    __shared__ int q_env[64], q_from[64];
    __shared__ int q_n;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t base = (int64_t)xcd_block(blockIdx.x, gridDim.x) * NENV;
    if (wv == 0) {
        const int64_t ev = base + lane;
        const bool ok = lane < NENV && ev < a.E;
        const int64_t evc = ok ? ev : a.E - 1;
        const uint32_t mw = a.mt_index[evc];
        const uint32_t rend = a.mt[evc * MT_WORDS + MT_RING_END];
        const int cnt = mi_cnt(mw), spar = mi_par(mw);
        const int from = cnt > 0 ? min((int)(rend & 0x3ffu), MT_N) + ((int)((rend >> 10) & 1u) != spar ? MT_N : 0)
                                 : min(mi_idx(mw), MT_N);
        const bool need = ok && from <= MT_N;
        const uint64_t M = __ballot(need);
        if (need) {
            const int k = mbcnt64(M);
            q_env[k] = lane;
            q_mw[k] = mw;
            q_rend[k] = rend;
            q_from[k] = from;
        }
        if (lane == 0) q_n = __popcll(M);
    }
    __syncthreads();
    const int n = __builtin_amdgcn_readfirstlane(q_n);
    for (int q = wv; q < n; q += NW) {
        const int64_t env = base + __builtin_amdgcn_readfirstlane(q_env[q]);
        const uint32_t mw = __builtin_amdgcn_readfirstlane(q_mw[q]);
        const uint32_t rend = __builtin_amdgcn_readfirstlane(q_rend[q]);
        const int from = __builtin_amdgcn_readfirstlane(q_from[q]);
        const uint32_t* src = a.mt + env * MT_WORDS + (uint32_t)mi_par(mw) * MT_ALT;
        uint32_t x[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) x[c] = (64 * c + lane < MT_N) ? src[64 * c + lane] : 0u;
        refill_env(a, env, mw, rend, from, x, lane);
    }
}

// ------------------------------------------------------- synthetic actions ---

__global__ void drl_synth_actions_kernel(uint64_t seed, uint64_t step, int64_t env_offset, int64_t total, int N,
                                         FastDiv dn, int fast, int32_t* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    uint64_t env, drone;
    if (fast) {  // total * N < 2^32: 32-bit multiply-shift division
        const uint32_t e = fdiv((uint32_t)t, dn);
        env = (uint64_t)(env_offset + e);
        drone = (uint32_t)t - e * (uint32_t)N;
    } else {
        env = (uint64_t)(env_offset + t / N);
        drone = (uint64_t)(t % N);
    }
    const uint64_t ctr = (step << 40) ^ (env << 8) ^ drone;
    const uint64_t h = splitmix64(seed ^ splitmix64(ctr));
    out[t] = (int32_t)(((h >> 32) * 5ull) >> 32);
}

// ---------------------------------------------------------------- launch ---
template <int P, class GEO>
static hipError_t launch_step_t(const StepArgs& a, hipStream_t s, int mode) {
    const int64_t blocks = (a.E + (64 / P) - 1) / (64 / P);
    const dim3 grid((unsigned)blocks), block(64);
    constexpr int WPB = step_wpb(P);  // drl_step_kernel's workgroups (the obs and rollout kernels: one wave)
    const dim3 sgrid((unsigned)((blocks + WPB - 1) / WPB)), sblock(64 * WPB);
    const size_t slds = WPB == 1 ? (size_t)a.wave_lds : (size_t)WPB * (size_t)((a.wave_lds + 15) & ~15);
    if (mode == kObsMode) {
        if constexpr (GEO::kObs) hipLaunchKernelGGL((drl_obs_kernel<P, GEO>), grid, block, a.wave_lds, s, a);
        else return hipErrorInvalidValue;
    } else if (mode == kRolloutMode) {
        if constexpr (P >= kRolloutNoObsMinLanes) hipLaunchKernelGGL((drl_rollout_kernel<P, GEO>), grid, block, a.wave_lds, s, a);
        else return hipErrorInvalidValue;
    } else if (GEO::kObs && a.code && a.ring_next) {  // drl_step_code_replay (no f32 observation)
        hipLaunchKernelGGL((drl_step_kernel<P, GEO, false, GEO::kObs, GEO::kObs>), sgrid, sblock, slds, s, a);
    } else if (GEO::kObs && a.code) {  // (obs NULL: the code alone)
        if (a.obs_nt) hipLaunchKernelGGL((drl_step_kernel<P, GEO, GEO::kObs, GEO::kObs>), sgrid, sblock, slds, s, a);
        else hipLaunchKernelGGL((drl_step_kernel<P, GEO, false, GEO::kObs>), sgrid, sblock, slds, s, a);
    } else if (GEO::kObs && a.obs && a.obs_nt) {
        hipLaunchKernelGGL((drl_step_kernel<P, GEO, GEO::kObs>), sgrid, sblock, slds, s, a);
    } else {
        hipLaunchKernelGGL((drl_step_kernel<P, GEO, false>), sgrid, sblock, slds, s, a);
    }
    return hipGetLastError();
}

// Compile-time-geometry instances for the benchmark shapes (side, drones,
// radius; observation of drone 0 or none), the runtime-geometry one otherwise.
template <int P, int G, int N, int R>
static bool launch_spec(const StepArgs& a, hipStream_t s, int mode, hipError_t* e) {
    if (a.side != G || a.n_drones != N || a.og.radius != R) return false;
    if (a.obs_k == 0 && mode != kObsMode) *e = launch_step_t<P, Geo<G, N, R, 0>>(a, s, mode);
    else if (a.obs_k == 1) *e = launch_step_t<P, Geo<G, N, R, 1>>(a, s, mode);
    else return false;
    return true;
}

hipError_t launch_step(const StepArgs& a, int P, hipStream_t s, int mode) {
    hipError_t e = hipSuccess;
    const bool spec = a.specialize;
    switch (P) {
        case 4:
            if (spec && launch_spec<4, 8, 4, 3>(a, s, mode, &e)) return e;
            return launch_step_t<4, GeoRT>(a, s, mode);
        case 8:
            if (spec && launch_spec<8, 16, 8, 3>(a, s, mode, &e)) return e;
            return launch_step_t<8, GeoRT>(a, s, mode);
        case 16:
            if (spec && launch_spec<16, 32, 16, 3>(a, s, mode, &e)) return e;
            return launch_step_t<16, GeoRT>(a, s, mode);
        case 32:
            if (spec && launch_spec<32, 64, 32, 3>(a, s, mode, &e)) return e;
            return launch_step_t<32, GeoRT>(a, s, mode);
        case 64: return launch_step_t<64, GeoRT>(a, s, mode);
        default: return hipErrorInvalidValue;
    }
}

#ifdef DRL_STAMPS
extern "C" int drl_debug_set_stamps(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_reset(const ResetArgs& a, hipStream_t s) {
    if (a.wave_per_env) {
        // waves (envs) per workgroup: 4 on large grids (C5 2.00e7 vs 1.91e7 resets/s), 1 below (C3 / C4 alike
        // within noise at 1, 2, 4; profiles/r04_reset/); DRL_RESET_WPB = 1, 2, 4 or 8 overrides (A/B knob)
        const int wpb = a.wpb ? a.wpb : (a.cells >= 4096 ? 4 : 1);
        const unsigned nb = (unsigned)((a.E + wpb - 1) / wpb);
        if (wpb == 8 && 8 * (size_t)a.wave_lds <= 160 * 1024)
            hipLaunchKernelGGL(drl_reset_wave_kernel<8>, dim3((unsigned)((a.E + 7) / 8)), dim3(512), 8 * (size_t)a.wave_lds, s, a);
        else if (wpb == 4 && 4 * (size_t)a.wave_lds <= 160 * 1024)
            hipLaunchKernelGGL(drl_reset_wave_kernel<4>, dim3(nb), dim3(256), 4 * (size_t)a.wave_lds, s, a);
        else if (wpb == 2 && 2 * (size_t)a.wave_lds <= 160 * 1024)
            hipLaunchKernelGGL(drl_reset_wave_kernel<2>, dim3(nb), dim3(128), 2 * (size_t)a.wave_lds, s, a);
        else
            hipLaunchKernelGGL(drl_reset_wave_kernel<1>, dim3((unsigned)a.E), dim3(64), a.wave_lds, s, a);
    } else {
        const int64_t blocks = (a.E + a.lanes - 1) / a.lanes;
        hipLaunchKernelGGL(drl_reset_kernel, dim3((unsigned)blocks), dim3(64), a.block_lds, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_decode(const uint32_t* drones, int64_t E, int N, int32_t* order, int32_t* y, int32_t* x,
                         int32_t* c, uint8_t* k, hipStream_t s) {
    const int64_t total = E * N;
    hipLaunchKernelGGL(drl_decode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, drones, total, N,
                       order, y, x, c, k);
    return hipGetLastError();
}

// packed grounds <-> a byte per cell (drl_env_get_state / drl_env_set_state)
__global__ void drl_ground_unpack_kernel(const uint8_t* __restrict__ packed, int pstride, uint8_t* __restrict__ out,
                                         int cells, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t e = i / cells;
    const int c = (int)(i - e * cells);
    out[i] = (uint8_t)nib_get(packed + e * pstride, c);
}
// (a code outside the ground objects {0, 2, 3, 4, 5} raises DRL_ERR_BAD_STATE: ADVICE r4)
__global__ void drl_ground_pack_kernel(const uint8_t* __restrict__ in, int cells, uint8_t* __restrict__ packed,
                                       int pstride, int64_t total, int32_t* __restrict__ err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one packed byte
    if (i >= total) return;
    const int64_t e = i / pstride;
    const int b = (int)(i - e * pstride), c0 = 2 * b;
    const uint8_t* row = in + e * cells;
    const uint32_t vlo = c0 < cells ? row[c0] : 0u, vhi = c0 + 1 < cells ? row[c0 + 1] : 0u;
    const auto bad = [](uint32_t v) { return v == 1u || v > 5u; };
    if (err && (bad(vlo) || bad(vhi))) atomicOr(err, DRL_ERR_BAD_STATE);
    packed[i] = (uint8_t)((vlo & 15u) | ((vhi & 15u) << 4));
}
hipError_t launch_ground_unpack(const uint8_t* packed, int pstride, uint8_t* out, int cells, int64_t E, hipStream_t s) {
    const int64_t total = E * cells;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(drl_ground_unpack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, packed, pstride,
                       out, cells, total);
    return hipGetLastError();
}
hipError_t launch_ground_pack(const uint8_t* in, int cells, uint8_t* packed, int pstride, int64_t E, int32_t* err,
                              hipStream_t s) {
    const int64_t total = E * pstride;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(drl_ground_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, cells, packed,
                       pstride, total, err);
    return hipGetLastError();
}

hipError_t launch_grid_obs(const uint8_t* ground, const uint32_t* drones, int64_t E, int side, int N, int gstride,
                           float* out, hipStream_t s) {
    hipLaunchKernelGGL(drl_grid_obs_kernel, dim3((unsigned)E), dim3(256), (size_t)side * side, s, ground, drones, side,
                       N, gstride, out);
    return hipGetLastError();
}

// Policy code -> observation (drl_code_decode): one thread per (row, cell),
// the channels of write_obs_wave from (object, air).
__global__ void __launch_bounds__(256) drl_code_decode_kernel(const uint16_t* __restrict__ code, int64_t n, int W,
                                                              int64_t code_stride, float* __restrict__ obs) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int cells = W * W;
    if (i >= n * cells) return;
    const int64_t row = i / cells;
    const int cl = (int)(i - row * cells);
    const int cpg = lay::code_cpg(W), cpg8 = lay::code_cpg8(W), grp = cl / cpg;
    const uint32_t h = code[row * code_stride + grp * cpg8 + (cl - grp * cpg)];
    const uint32_t obj = h & 7u, air = h >> 3;
    float2* o = reinterpret_cast<float2*>(obs + i * 6);
    o[0] = make_float2(air ? 1.0f : 0.0f, (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f);
    o[1] = make_float2(obj == OBJ_DROPZONE ? 1.0f : 0.0f, obj == OBJ_STATION ? 1.0f : 0.0f);
    o[2] = make_float2(air ? div100((int)(air & 0x7fu) - 1) : 0.0f, obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f);
}

hipError_t launch_code_decode(const void* code, int64_t n, int W, float* obs, hipStream_t s) {
    const int64_t total = n * W * W;
    hipLaunchKernelGGL(drl_code_decode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       static_cast<const uint16_t*>(code), n, W, (int64_t)(lay::code_bytes(W) / 2), obs);
    return hipGetLastError();
}

// ------------------------------------------------------------ HBM probe ---
// SURVEY.md §8 D3's "measured copy-kernel" peak beside the 8 TB/s spec
// (drl_hbm_probe): the plain grid-sized float4 copy of MI355X_MICROARCH.md's
// 6.29 TB/s figure -- one 16-B element per lane, ordinary loads and stores, a
// grid covering the buffer.  The read form folds each element into a compare
// whose (practically never taken) store stays inside dst's first `bytes`.
template <bool COPY>
__global__ void __launch_bounds__(256) drl_hbm_probe_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                            int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u32x4 v = src[i];
    if constexpr (COPY) {
        dst[i] = v;
    } else {
        if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) dst[i].x = v.x;
    }
}

hipError_t launch_hbm_probe(const void* src, void* dst, int64_t bytes, int mode, int num_cus, hipStream_t s) {
    (void)num_cus;
    const int64_t n = bytes / 16;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (mode == 0)
        hipLaunchKernelGGL(drl_hbm_probe_kernel<true>, grid, dim3(256), 0, s, static_cast<const u32x4*>(src),
                           static_cast<u32x4*>(dst), n);
    else
        hipLaunchKernelGGL(drl_hbm_probe_kernel<false>, grid, dim3(256), 0, s, static_cast<const u32x4*>(src),
                           static_cast<u32x4*>(dst), n);
    return hipGetLastError();
}

hipError_t launch_encode(uint32_t* drones, int64_t E, int N, const int32_t* order, const int32_t* y,
                         const int32_t* x, const int32_t* c, const uint8_t* k, hipStream_t s) {
    const int64_t total = E * N;
    hipLaunchKernelGGL(drl_encode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, drones, total, N,
                       order, y, x, c, k);
    return hipGetLastError();
}

hipError_t launch_refill(const RefillArgs& a, hipStream_t s) {
    if (a.list) {
        hipLaunchKernelGGL((drl_refill_list_kernel<kRefillListEnvs, kRefillListWaves>),
                           dim3((unsigned)((a.E + kRefillListEnvs - 1) / kRefillListEnvs)), dim3(64 * kRefillListWaves),
                           0, s, a);
        return hipGetLastError();
    }
    const int64_t blocks = (a.E + kRefillWaves * kRefillEnvs - 1) / (kRefillWaves * kRefillEnvs);
    hipLaunchKernelGGL(drl_refill_kernel, dim3((unsigned)blocks), dim3(64 * kRefillWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_mt_get(const uint32_t* mt, const uint32_t* mt_index, int64_t E, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(drl_mt_get_kernel, dim3((unsigned)((E * 625 + 255) / 256)), dim3(256), 0, s, mt, mt_index, E, out);
    return hipGetLastError();
}

hipError_t launch_mt_set(uint32_t* mt, uint32_t* mt_index, int64_t E, const uint32_t* in, int32_t* err, hipStream_t s) {
    hipLaunchKernelGGL(drl_mt_set_kernel, dim3((unsigned)((E * 625 + 255) / 256)), dim3(256), 0, s, mt, mt_index, E, in,
                       err);
    return hipGetLastError();
}

hipError_t launch_synth(uint64_t seed, uint64_t step, int64_t env_offset, int64_t E, int N, int32_t* out,
                        hipStream_t s) {
    const int64_t total = E * N;
    const int fast = (uint64_t)total * (uint64_t)N < (1ull << 32) ? 1 : 0;
    hipLaunchKernelGGL(drl_synth_actions_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, seed, step,
                       env_offset, total, N, make_fastdiv((uint32_t)N), fast, out);
    return hipGetLastError();
}

}  // namespace drl
