// dronerl_kernels.hip — batched DroneRL env kernels for MI355X (gfx950, CDNA4).
//
// Semantics: nyx-ai/droneRL torch_impl (env.py:68-233, wrappers.py:10-73),
// bit-exact including each env's CPython MT19937 draw stream.  Layout and
// design: DESIGN.md.  Summary:
//
//  drl_step_kernel<P>  one wavefront lane per (env, drone slot); an env owns a
//      group of P lanes (P = pow2 >= n_drones), 64/P envs per wave, 4 waves
//      per block.  Slots are kept in dict order O, so "earlier in O" is "lower
//      lane".  The env's ground is staged into LDS with 16-B vector copies,
//      first-comer claims / crash ordering are resolved with __shfl/__ballot,
//      and the serial respawn section (env.py:186-210) draws P MT outputs per
//      round in parallel and picks the first accepted (y, x) pair with ballots.
//      The observation window is written from LDS with 16-B stores.
//  drl_obs_kernel<P>   the same geometry, observation only.
//  drl_reset_kernel    one lane per env (64-lane blocks): the reset is a long
//      serial shuffle/sample chain per env (env.py:68-101); the shuffle list
//      lives in LDS, MT twists are done cooperatively by the whole wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronerl_internal.h"

namespace drl {

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

// In-place MT19937 twist of one env's state by all 64 lanes of the wave,
// register-resident: lane l holds x[c] = mt[64c + l].  Chunks are processed in
// ascending order, each computed from old/new values exactly as the sequential
// generator sees them: mt[i+1] and mt[i+397] (i < 227) are still old (chunks
// > c), mt[i-227] (i >= 227) and mt[0] (i = 623) are already new (chunks < c).
// Lane offsets are constants (397 = 6*64 + 13, 227 = 4*64 - 29).
__device__ __noinline__ void twist_wave(uint32_t* row, int lane) {
    uint32_t x[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int i = 64 * c + lane;
        x[c] = (i < MT_N) ? load_l2(row + i) : 0u;
    }
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int i = 64 * c + lane;
        uint32_t nxt = __shfl(x[c], (lane + 1) & 63);
        if (c < 9) {
            const uint32_t n0 = __shfl(x[c + 1], 0);
            if (lane == 63) nxt = n0;
        } else {
            const uint32_t m0 = __shfl(x[0], 0);  // new mt[0]
            if (i == MT_N - 1) nxt = m0;
        }
        const int l13 = lane + 13, l29 = lane + 29;
        const uint32_t fo_a = (c + 6 < 10) ? __shfl(x[(c + 6) % 10], l13 & 63) : 0u;
        const uint32_t fo_b = (c + 7 < 10) ? __shfl(x[(c + 7) % 10], l13 & 63) : 0u;
        const uint32_t fn_a = (c >= 4) ? __shfl(x[(c + 6) % 10], l29 & 63) : 0u;  // x[c-4]
        const uint32_t fn_b = (c >= 3) ? __shfl(x[(c + 7) % 10], l29 & 63) : 0u;  // x[c-3]
        const uint32_t far = (i < MT_N - MT_M) ? (l13 < 64 ? fo_a : fo_b) : (l29 < 64 ? fn_a : fn_b);
        const uint32_t y = (x[c] & 0x80000000u) | (nxt & 0x7fffffffu);
        x[c] = far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
#pragma unroll
    for (int c = 0; c < 10; ++c) {
        const int i = 64 * c + lane;
        if (i < MT_N) row[i] = x[c];
    }
    // make the rewritten words visible to this workgroup's later sc1 loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
}

// ------------------------------------------------------- observation write ---
// Per-wave LDS image of its envs (every region a multiple of 16 B):
//   gl  [GPW][gstride] ground codes      al [GPW][gstride] air: 0 or (charge+1)|carry<<7
//   mtw [GPW][PF] u32  prefetched MT words   posidx [GPW][NP] u16 cell of drone index k
struct WaveLds {
    uint8_t* gl;
    uint8_t* al;
    uint32_t* mtw;
    uint16_t* posidx;
};

__device__ __forceinline__ WaveLds carve(unsigned char* wbase, int gpw, int gstride, int np) {
    WaveLds w;
    w.gl = wbase;
    w.al = w.gl + gpw * gstride;
    w.mtw = reinterpret_cast<uint32_t*>(w.al + gpw * gstride);
    w.posidx = reinterpret_cast<uint16_t*>(w.mtw + gpw * MT_PF);
    (void)np;
    return w;
}

// WindowedGridView windows (wrappers.py:10-31,55-73) of the wave's envs:
// lane = one window cell; its 6 channels are computed branch-free and stored
// as three 8-B pieces (consecutive lanes cover a contiguous span).  ch0 drone,
// ch1 packet OR carrying drone, ch2 dropzone, ch3 station, ch4 charge/100
// (true f32 division, == f32(double c/100)), ch5 skyscraper or wall.
__device__ __forceinline__ void write_obs_wave(float* __restrict__ obs, int64_t wenv0, int nenv_w,
                                               const ObsGeom& g, const WaveLds& w, int np, int lane) {
    const uint32_t win = g.W * g.W;
    const uint32_t env_cells = g.env_floats / 6u;  // K * W*W
    const uint32_t ncell = (uint32_t)nenv_w * env_cells;
    float* base = obs + wenv0 * (int64_t)g.env_floats;
    for (uint32_t q = lane; q < ncell; q += 64) {
        const uint32_t e = fdiv(q, g.div_env);
        uint32_t rem = q - e * env_cells;
        const uint32_t k = fdiv(rem, g.div_per);
        rem -= k * win;
        const uint32_t wy = fdiv(rem, g.div_w);
        const uint32_t wx = rem - wy * g.W;
        const uint32_t pos = w.posidx[e * np + k];
        const uint32_t py = fdiv(pos, g.div_side);
        const uint32_t px = pos - py * (uint32_t)g.side;
        const int y = (int)(py + wy) - g.radius;
        const int x = (int)(px + wx) - g.radius;
        const bool in = (unsigned)y < (unsigned)g.side && (unsigned)x < (unsigned)g.side;
        const uint32_t cell = e * g.gstride + (uint32_t)(y * g.side + x);
        const uint32_t obj = in ? w.gl[cell] : (uint32_t)OBJ_SKYSCRAPER;
        const uint32_t air = in ? w.al[cell] : 0u;
        float2 v01, v23, v45;
        v01.x = air ? 1.0f : 0.0f;
        v01.y = (obj == OBJ_PACKET || (air & 0x80u)) ? 1.0f : 0.0f;
        v23.x = obj == OBJ_DROPZONE ? 1.0f : 0.0f;
        v23.y = obj == OBJ_STATION ? 1.0f : 0.0f;
        v45.x = air ? (float)((int)(air & 0x7fu) - 1) / 100.0f : 0.0f;
        v45.y = obj == OBJ_SKYSCRAPER ? 1.0f : 0.0f;
        float2* o = reinterpret_cast<float2*>(base + 6u * q);
        o[0] = v01;
        o[1] = v23;
        o[2] = v45;
    }
}

// Stage a wave's grounds (contiguous, env-major) into LDS and clear the air map.
__device__ __forceinline__ void stage_ground(const uint8_t* __restrict__ ground, int64_t wenv0, int nenv_w,
                                             int gstride, const WaveLds& w, int lane) {
    const uint4* src = reinterpret_cast<const uint4*>(ground + wenv0 * gstride);
    const int nvec = nenv_w * gstride / 16;
    for (int v = lane; v < nvec; v += 64) {
        reinterpret_cast<uint4*>(w.gl)[v] = src[v];
        reinterpret_cast<uint4*>(w.al)[v] = make_uint4(0u, 0u, 0u, 0u);
    }
}

// ------------------------------------------------------------------ step ---
template <int P>
__global__ void __launch_bounds__(256) drl_step_kernel(StepArgs a) {
    constexpr int GPW = 64 / P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = lane / P;
    const int j = lane % P;
    const int64_t wenv0 = ((int64_t)blockIdx.x * a.wpb + wave) * GPW;
    const int nenv_w = (int)min((int64_t)GPW, a.E - wenv0);
    if (nenv_w <= 0) return;  // no block-level barriers anywhere: whole idle waves may leave
    const int64_t env = wenv0 + grp;
    const bool env_ok = grp < nenv_w;
    const int G = a.side, N = a.n_drones, gstride = a.gstride, np = a.np;
    const WaveLds W = carve(smem + wave * a.wave_lds, GPW, gstride, np);
    uint8_t* gl = W.gl + grp * gstride;
    uint8_t* al = W.al + grp * gstride;
    uint32_t* mtw = W.mtw + grp * MT_PF;
    uint16_t* posidx = W.posidx + grp * np;

    // ---- loads, all independent: drone record, this lane's action (by drone
    // index j), the env's MT index, the ground (-> LDS)
    const bool active = env_ok && j < N;
    const uint32_t rec = active ? a.drones[env * N + j] : 0u;
    const int my_action = active ? a.actions[env * N + j] : 4;
    const uint32_t* mrow = a.mt + (env_ok ? env : 0) * MT_WORDS;
    int midx = env_ok ? (int)mrow[MT_N] : MT_N;
    stage_ground(a.ground, wenv0, nenv_w, gstride, W, lane);
    // prefetch the next MT_PF words of the stream into LDS (dependent on midx only)
    const int pf_base0 = midx;
    int pfn = min(MT_PF, MT_N - midx);
    for (int o = j; o < pfn; o += P) mtw[o] = mrow[midx + o];

    const int y = rec & 255u, x = (rec >> 8) & 255u;
    const int idx = ((int)(rec >> 25) < N) ? (int)(rec >> 25) : j;  // corrupt records never index out of bounds
    int c = (rec >> 16) & 255u;
    int carry = (rec >> 24) & 1u;
    int act = __shfl(my_action, idx, P);  // actions are by drone index (env.py:125)
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
    const int tcell = inb ? ty * G + tx : -1;

    // ---- phase 1 claims (env.py:124-140): first in O order claims a cell;
    // later ones crash (list A) and record the cell; OOB crashes (list A).
    bool earlier = false;
    int later_min = P;
#pragma unroll
    for (int s = 0; s < P; ++s) {
        const int ts = __shfl(tcell, s, P);
        if (inb && ts == tcell) {
            if (s < j) earlier = true;
            else if (s > j && s < later_min) later_min = s;
        }
    }
    const bool claimer = inb && !earlier;
    const bool crashA = active && !claimer;
    wave_sync();

    // ---- phase 2 effects on claimers (env.py:143-172), own cell only
    float reward = 0.0f;
    bool dead = false, deliver = false, dirty = false;
    if (claimer) {
        const int obj = gl[tcell];
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
            gl[tcell] = OBJ_EMPTY;
            dirty = true;
        } else if (obj == OBJ_DROPZONE && carry) {
            reward = a.r_delivery;
            carry = 0;
            gl[tcell] = OBJ_EMPTY;
            deliver = true;
            dirty = true;
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
    const uint64_t gm = (P == 64) ? ~0ull : (((1ull << P) - 1ull) << gshift);
    const uint64_t lower = (1ull << lane) - 1ull;
    const uint64_t bS = __ballot(survivor) & gm;
    const uint64_t bA = __ballot(crashA) & gm;
    const uint64_t bB = __ballot(crashB) & gm;
    const int nS = __popcll(bS), nA = __popcll(bA), nR = nA + __popcll(bB);
    int rankB = 0;
    if (bB) {
        const int bkey = crashB ? (collided ? later_min : P + j) : 4 * P;
#pragma unroll
        for (int s = 0; s < P; ++s) rankB += (__shfl(bkey, s, P) < bkey);
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
    if (survivor) al[tcell] = 1;
    bool gdirty = (__ballot(dirty) & gm) != 0ull;
    wave_sync();

    // ---- respawns (env.py:186-210, _find_respawn_position :226-233):
    // items w < nR: crashed drones (mask: drones | skyscrapers); then n_pack
    // packets, then n_deliver dropzones (mask: any ground object).  Each round
    // draws P consecutive MT outputs, keeps those < side (randint(0, side-1)
    // == _randbelow(side)), pairs accepted draws as (y, x) and takes the
    // first pair whose cell is free.
    int pf_base = pf_base0;
    int w = 0, have_y = 0, yv = 0;
    const int shift = 32 - a.kbits;
    uint32_t rounds = 0;
    for (;;) {
        const bool work = env_ok && w < total;
        if (!__ballot(work)) break;
        uint64_t need = __ballot(work && j == 0 && midx >= MT_N);
        while (need) {
            const int tl = __ffsll((unsigned long long)need) - 1;
            need &= need - 1ull;
            twist_wave(a.mt + (wenv0 + tl / P) * MT_WORDS, lane);
            if (grp == tl / P) {
                midx = 0;
                pf_base = 0;
                pfn = 0;  // prefetched words are stale now
            }
        }
        if (work) {
            const int avail = MT_N - midx;
            const bool valid = j < avail;
            const int off = midx - pf_base + j;
            uint32_t word = 0u;
            if (valid) word = (off < pfn) ? mtw[off] : load_l2(mrow + midx + j);
            const int r = valid ? (int)(temper(word) >> shift) : G;
            const bool acc = valid && r < G;
            const uint64_t accb = (__ballot(acc) & gm) >> gshift;
            const uint64_t lowrel = (1ull << j) - 1ull;
            const int apos = have_y + __popcll(accb & lowrel);
            const uint64_t prevm = accb & lowrel;
            const int prevlane = prevm ? 63 - __clzll((long long)prevm) : 0;
            const int rprev = __shfl(r, prevlane, P);
            const int ycand = prevm ? rprev : yv;
            const bool cand = acc && (apos & 1);
            const int ccell = ycand * G + r;
            bool free_cell = false;
            if (cand) {
                const int obj = gl[ccell];
                free_cell = (w < nR) ? (al[ccell] == 0 && obj != OBJ_SKYSCRAPER) : (obj == OBJ_EMPTY);
            }
            const uint64_t okb = (__ballot(cand && free_cell) & gm) >> gshift;
            if (okb) {
                const int js = __ffsll((unsigned long long)okb) - 1;
                const int cell = __shfl(ccell, js, P);
                if (w < nR) {
                    if (crashed && newslot == nS + w) pos = cell;
                    if (j == 0) al[cell] = 1;
                } else {
                    if (j == 0) gl[cell] = (w < nR + n_pack) ? OBJ_PACKET : OBJ_DROPZONE;
                    gdirty = true;
                }
                midx += js + 1;
                ++w;
                have_y = 0;
            } else {
                const int cnt = have_y + __popcll(accb);
                if (accb && (cnt & 1)) yv = __shfl(r, 63 - __clzll((long long)accb), P);
                have_y = cnt & 1;
                midx += min(P, avail);
            }
            if (++rounds > a.max_rounds) {  // full grid: the reference spins forever
                if (j == 0 && a.err) atomicOr(a.err, DRL_ERR_NO_FREE_CELL);
                w = total;
                if (crashed && pos < 0) pos = 0;
            }
        }
        wave_sync();
    }

    // ---- _pick_packets_after_respawn (env.py:217-224): distinct cells, parallel
    if (active && pos < 0) pos = 0;  // unreachable for valid params (respawn always finds a cell)
    if (active && !carry && gl[pos] == OBJ_PACKET) {
        carry = 1;
        gl[pos] = OBJ_EMPTY;
        dirty = true;
    }
    gdirty |= (__ballot(dirty) & gm) != 0ull;

    // ---- write back: records permuted to O', rewards/dones by drone index
    if (active) {
        const uint32_t py = fdiv((uint32_t)pos, a.div_side);
        const uint32_t px = (uint32_t)pos - py * (uint32_t)G;
        a.drones[env * N + newslot] = pack_drone((int)py, (int)px, c, carry, idx);
        a.rewards[env * N + idx] = reward;
        a.dones[env * N + idx] = crashed ? 1 : 0;
        posidx[idx] = (uint16_t)pos;
        al[pos] = (uint8_t)((c + 1) | (carry << 7));
    }
    if (env_ok && j == 0) a.mt[env * MT_WORDS + MT_N] = (uint32_t)midx;
    wave_sync();
    if (env_ok && gdirty) {
        uint4* dst = reinterpret_cast<uint4*>(a.ground + env * gstride);
        const uint4* src = reinterpret_cast<const uint4*>(gl);
        for (int v = j; v < gstride / 16; v += P) dst[v] = src[v];
    }
    if (a.obs) write_obs_wave(a.obs, wenv0, nenv_w, a.og, W, np, lane);
}

// ------------------------------------------------------------ observation ---
template <int P>
__global__ void __launch_bounds__(256) drl_obs_kernel(StepArgs a) {
    constexpr int GPW = 64 / P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = lane / P;
    const int j = lane % P;
    const int64_t wenv0 = ((int64_t)blockIdx.x * a.wpb + wave) * GPW;
    const int nenv_w = (int)min((int64_t)GPW, a.E - wenv0);
    if (nenv_w <= 0) return;
    const int64_t env = wenv0 + grp;
    const bool env_ok = grp < nenv_w;
    const int N = a.n_drones, gstride = a.gstride, np = a.np;
    const WaveLds W = carve(smem + wave * a.wave_lds, GPW, gstride, np);
    stage_ground(a.ground, wenv0, nenv_w, gstride, W, lane);
    wave_sync();
    if (env_ok && j < N) {
        const uint32_t rec = a.drones[env * N + j];
        const int pos = (int)(rec & 255u) * a.side + (int)((rec >> 8) & 255u);
        const int c = (rec >> 16) & 255u, carry = (rec >> 24) & 1u;
        const int idx = ((int)(rec >> 25) < N) ? (int)(rec >> 25) : j;
        W.posidx[grp * np + idx] = (uint16_t)pos;
        W.al[grp * gstride + pos] = (uint8_t)((c + 1) | (carry << 7));
    }
    wave_sync();
    write_obs_wave(a.obs, wenv0, nenv_w, a.og, W, np, lane);
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

__global__ void __launch_bounds__(64) drl_reset_kernel(ResetArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int64_t env = (int64_t)blockIdx.x * a.lanes + lane;
    const bool own = lane < a.lanes && env < a.E && (a.mask == nullptr || a.mask[env] != 0);
    uint16_t* list = reinterpret_cast<uint16_t*>(smem + (size_t)lane * a.lane_lds);
    uint16_t* sel = list + a.list_cap;
    uint16_t* pool = sel + 64;
    const int GG = a.cells, N = a.n_drones;
    uint32_t* mrow = a.mt + (own ? env : 0) * MT_WORDS;
    uint8_t* grow = a.ground + (own ? env : 0) * a.gstride;

    if (own) {
        if (a.reseed) mt_seed_row(mrow, a.seed_base + (uint64_t)env);
        for (int v = 0; v < a.gstride / 16; ++v) reinterpret_cast<uint4*>(grow)[v] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = 0; i < GG; ++i) list[i] = (uint16_t)i;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int midx = own ? (a.reseed ? MT_N : (int)mrow[MT_N]) : MT_N;
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
            twist_wave(a.mt + ((int64_t)blockIdx.x * a.lanes + tl_) * MT_WORDS, lane);     \
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
        for (int t = 0; t < a.n_sky; ++t) grow[list[n - 1 - t]] = OBJ_SKYSCRAPER;
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
        for (int t = 0; t < a.n_pack; ++t) grow[list[n - 1 - t]] = OBJ_PACKET;
    n -= a.n_pack;
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_drop; ++t) grow[list[n - 1 - t]] = OBJ_DROPZONE;
    n -= a.n_drop;
    DRL_SHUFFLE(n)
    if (own)
        for (int t = 0; t < a.n_stat; ++t) grow[list[n - 1 - t]] = OBJ_STATION;
    n -= a.n_stat;
#undef DRL_SHUFFLE
#undef DRL_DRAW_LOOP

    // drones in index order (dict order 0..N-1), then _pick_packets_after_respawn
    if (own) {
        for (int d = 0; d < N; ++d) {
            const int cell = sel[d];
            int carry = 0;
            if (grow[cell] == OBJ_PACKET) {
                carry = 1;
                grow[cell] = OBJ_EMPTY;
            }
            const uint32_t py = fdiv((uint32_t)cell, a.div_side);
            a.drones[env * N + d] = pack_drone((int)py, cell - (int)py * a.side, 100, carry, d);
        }
        mrow[MT_N] = (uint32_t)midx;
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

// ------------------------------------------------------- synthetic actions ---
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ void drl_synth_actions_kernel(uint64_t seed, uint64_t step, int64_t env_offset, int64_t total, int N,
                                         int32_t* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const uint64_t env = (uint64_t)(env_offset + t / N);
    const uint64_t drone = (uint64_t)(t % N);
    const uint64_t ctr = (step << 40) ^ (env << 8) ^ drone;
    const uint64_t h = splitmix64(seed ^ splitmix64(ctr));
    out[t] = (int32_t)(((h >> 32) * 5ull) >> 32);
}

// ---------------------------------------------------------------- launch ---
template <int P>
static hipError_t launch_step_t(const StepArgs& a, hipStream_t s, bool obs_only) {
    const int envs_per_block = a.wpb * (64 / P);
    const int64_t blocks = (a.E + envs_per_block - 1) / envs_per_block;
    const dim3 grid((unsigned)blocks), block(64 * a.wpb);
    if (obs_only)
        hipLaunchKernelGGL(drl_obs_kernel<P>, grid, block, a.wpb * a.wave_lds, s, a);
    else
        hipLaunchKernelGGL(drl_step_kernel<P>, grid, block, a.wpb * a.wave_lds, s, a);
    return hipGetLastError();
}

hipError_t launch_step(const StepArgs& a, int P, hipStream_t s, bool obs_only) {
    switch (P) {
        case 4: return launch_step_t<4>(a, s, obs_only);
        case 8: return launch_step_t<8>(a, s, obs_only);
        case 16: return launch_step_t<16>(a, s, obs_only);
        case 32: return launch_step_t<32>(a, s, obs_only);
        case 64: return launch_step_t<64>(a, s, obs_only);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_reset(const ResetArgs& a, hipStream_t s) {
    const int64_t blocks = (a.E + a.lanes - 1) / a.lanes;
    hipLaunchKernelGGL(drl_reset_kernel, dim3((unsigned)blocks), dim3(64), a.block_lds, s, a);
    return hipGetLastError();
}

hipError_t launch_decode(const uint32_t* drones, int64_t E, int N, int32_t* order, int32_t* y, int32_t* x,
                         int32_t* c, uint8_t* k, hipStream_t s) {
    const int64_t total = E * N;
    hipLaunchKernelGGL(drl_decode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, drones, total, N,
                       order, y, x, c, k);
    return hipGetLastError();
}

hipError_t launch_encode(uint32_t* drones, int64_t E, int N, const int32_t* order, const int32_t* y,
                         const int32_t* x, const int32_t* c, const uint8_t* k, hipStream_t s) {
    const int64_t total = E * N;
    hipLaunchKernelGGL(drl_encode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, drones, total, N,
                       order, y, x, c, k);
    return hipGetLastError();
}

hipError_t launch_synth(uint64_t seed, uint64_t step, int64_t env_offset, int64_t E, int N, int32_t* out,
                        hipStream_t s) {
    const int64_t total = E * N;
    hipLaunchKernelGGL(drl_synth_actions_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, seed, step,
                       env_offset, total, N, out);
    return hipGetLastError();
}

}  // namespace drl
