// dronerl_api.cpp — the C ABI (include/dronerl.h): parameter validation,
// launch geometry, error reporting.  No allocation, no synchronisation.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "dronerl_internal.h"

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

int hip_fail(hipError_t e, const char* what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -2;
}

int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

int bit_length(uint32_t n) {
    int k = 0;
    while (n) { ++k; n >>= 1; }
    return k;
}

constexpr int kStepLdsTarget = 64 * 1024;   // per block
constexpr int kLdsMax = 160 * 1024;
constexpr int kResetLdsTarget = 64 * 1024;
constexpr int kFySerial = 4;    // reset (wave kernel): i-range writers per chunk resolved serially
constexpr int kFyBatchMin = 1;  // reset (wave kernel): shuffle 64 draws at a time down to si = 1 (measured best)

using drl::lay::r16;
int env_np(int n_drones) { return drl::lay::np(n_drones); }

// Per-env LDS regions of drl_step (see WaveLds in dronerl_kernels.hip)
struct EnvLds {
    int bm, paint, chg, nchg, fixed, scratch;
};
EnvLds env_lds(int gstride, int cells, int n_drones, int obs_k, int window, int P) {
    EnvLds e;
    e.bm = drl::lay::bm_bytes(cells);
    e.paint = drl::lay::paint_bytes(obs_k, window);
    e.nchg = drl::lay::nchg(n_drones);
    e.chg = drl::lay::chg_bytes(n_drones);
    e.fixed = gstride + e.paint + 2 * env_np(n_drones);
    e.scratch = e.bm + 4 * P + e.chg + 16;  // 4 * P: the rollout's record stash
    return e;
}

// LDS bytes per wave of drl_step: per-env regions + the scratch area, which
// must also hold the observation transpose stage.
int wave_lds_bytes(int gpw, const EnvLds& e, bool obs) {
    int scratch = gpw * e.scratch;
    if (obs && scratch < drl::OBS_U * 1536) scratch = drl::OBS_U * 1536;
    return gpw * e.fixed + scratch;
}

// lanes per env in drl_step: pow2 >= n_drones (>= 4), widened when one wave
// of narrower groups would not fit a quarter of the LDS target.
int step_group_lanes(int n_drones, int gstride, int cells, int window) {
    int P = 1;
    while (P < (n_drones < 4 ? 4 : n_drones)) P <<= 1;
    while (P < 64 && wave_lds_bytes(64 / P, env_lds(gstride, cells, n_drones, 1, window, P), true) > kStepLdsTarget / 4)
        P <<= 1;
    return P;
}

// Steps between refills.  A refill converts a whole MT block into ring
// entries once an env's stream has moved into the block the ring ends in, so
// the ring then holds that block's remaining entries: 312 * side / 2^kbits
// pairs per block (_randbelow's acceptance; 156 at power-of-two sides).  Ring
// entries used per env-step, measured at the benchmark shapes with random
// actions (tools/ring_usage.py): mean 2.06 / 2.56 / 3.44 and at most 17 at N =
// 8 / 16 / 32, i.e. about 1.53 + 0.06 N, and up to ~2.2x the mean over 16
// steps.  A refill every half block's worth of mean use (at most 32 steps)
// keeps the heaviest envs off the dry-ring path.  Round 4 (block-conversion
// refill, profiles/r04_refill/): 0.62 of a block's mean use, capped at 48 --
// 48 at C3 (3.24-3.25e9 env-steps/s against 3.20e9 at 32 and 3.19e9 at 64),
// 38 at C4, 28 at C5 (22, 32: 9.07-9.11e8 alike, 44: 8.98e8).
// The bytes per step do not depend on the cadence (each block is converted
// once); only the launch count and the dry-ring risk do.  DRL_REFILL_EVERY
// overrides it (A/B runs) with a positive step count; anything else is
// refused (0 would read as "never" in the Python env's refill_every, ADVICE
// r2), and the cadence stays >= 1 for drl_rollout's narrow-group modulo.
int refill_cadence(int n_drones, int side) {
    if (const char* v = getenv("DRL_REFILL_EVERY")) {
        char* end = nullptr;
        const long r = strtol(v, &end, 10);
        return (end != v && *end == 0 && r > 0 && r <= 1 << 20) ? (int)r : -1;
    }
    const double per_block = (DRL_MT_BLOCK1 / 2.0) * side / (double)(1 << bit_length((uint32_t)side));
    const int r = (int)(0.62 * per_block / (1.53 + 0.06 * n_drones));
    return r < 1 ? 1 : (r > 48 ? 48 : r);
}

int validate(const drl_params* p, drl_layout* L) {
    if (!p) return fail("params is NULL");
    if (p->side < 2 || p->side > DRL_MAX_SIDE) return fail("side %d outside [2, %d]", p->side, DRL_MAX_SIDE);
    if (p->n_drones < 1 || p->n_drones > DRL_MAX_DRONES)
        return fail("n_drones %d outside [1, %d]", p->n_drones, DRL_MAX_DRONES);
    if (p->charge < 0 || p->discharge < 0) return fail("charge/discharge must be >= 0");
    if (p->window_radius < 1 || p->window_radius > DRL_MAX_RADIUS)
        return fail("window_radius %d outside [1, %d]", p->window_radius, DRL_MAX_RADIUS);
    if (p->packets_factor < 0 || p->dropzones_factor < 0 || p->stations_factor < 0 || p->skyscrapers_factor < 0)
        return fail("object factors must be >= 0");
    const int GG = p->side * p->side, N = p->n_drones;
    const long sky = (long)p->skyscrapers_factor * N, pack = (long)p->packets_factor * N;
    const long drop = (long)p->dropzones_factor * N, stat = (long)p->stations_factor * N;
    // spawn_objects (env.py:59-60) and Random.sample ValueErrors
    if (sky > GG) return fail("Not enough positions (%d) to spawn %ld objects", GG, sky);
    if (N > GG - sky) return fail("Sample larger than population or is negative");
    if (sky + pack + drop + stat > GG)
        return fail("Not enough positions (%ld) to spawn %ld objects", GG - sky, pack + drop + stat);
    if (L) {
        L->side = p->side;
        L->n_drones = N;
        L->cells = GG;
        L->ground_stride = drl::lay::pstride(p->side);  // packed nibbles (the LDS image: 2x, lay::gstride)
        L->drone_stride = N;
        L->mt_stride = DRL_MT_WORDS;
        L->obs_window = 2 * p->window_radius + 1;
        L->obs_floats = L->obs_window * L->obs_window * 6;
        const int lg = drl::lay::glstride(p->side);  // LDS ground bytes per env
        L->step_group_lanes = step_group_lanes(N, lg, GG, L->obs_window);
        L->step_lds_bytes =
            wave_lds_bytes(64 / L->step_group_lanes, env_lds(lg, GG, N, 1, L->obs_window, L->step_group_lanes), true);
        if (L->step_lds_bytes > kLdsMax) return fail("side %d needs %d B of LDS per block", p->side, L->step_lds_bytes);
        L->cand_slots = DRL_CAND_SLOTS;
        L->refill_every = refill_cadence(N, p->side);
        if (L->refill_every < 1) return fail("DRL_REFILL_EVERY must be a positive integer step count");
    }
    return 0;
}

int check_state(const drl_state* s, const drl_layout& L) {
    if (!s) return fail("state is NULL");
    if (s->num_envs < 0) return fail("num_envs < 0");
    if (s->num_envs > 0 && (!s->ground || !s->drones || !s->mt || !s->mt_index)) return fail("state has NULL buffers");
    if ((uintptr_t)s->ground % 16) return fail("ground must be 16-byte aligned");
    (void)L;
    return 0;
}

drl::ObsGeom obs_geom(const drl_params* p, const drl_layout& L, int k) {
    drl::ObsGeom g;
    g.side = p->side;
    g.radius = p->window_radius;
    g.W = (uint32_t)L.obs_window;
    g.per = (uint32_t)L.obs_floats;
    g.env_floats = (uint32_t)(k > 0 ? k : 1) * g.per;
    g.gstride = (uint32_t)drl::lay::glstride(p->side);
    g.div_env = drl::make_fastdiv(g.env_floats / 6u);  // window cells per env
    g.div_per = drl::make_fastdiv(g.W * g.W);          // cells per window
    g.div_6 = drl::make_fastdiv(6);
    g.div_w = drl::make_fastdiv(g.W);
    g.div_side = drl::make_fastdiv((uint32_t)p->side);
    return g;
}

drl::StepArgs step_args(const drl_params* p, const drl_state* s, const drl_layout& L, int obs_k) {
    drl::StepArgs a;
    memset(&a, 0, sizeof a);
    a.side = p->side;
    a.n_drones = p->n_drones;
    a.gstride = drl::lay::glstride(p->side);  // LDS (a byte per cell, or the packed HBM row: lay::gl_nib)
    a.pstride = drl::lay::pstride(p->side);
    a.gl_nib = drl::lay::gl_nib(p->side) ? 1 : 0;
    a.kbits = bit_length((uint32_t)p->side);
    a.charge = p->charge;
    a.discharge = p->discharge;
    a.r_pickup = p->pickup_reward;
    a.r_delivery = p->delivery_reward;
    a.r_crash = p->crash_reward;
    a.r_charge = p->charge_reward;
    a.E = s->num_envs;
    a.ground = s->ground;
    a.drones = s->drones;
    a.mt = s->mt;
    a.mt_index = s->mt_index;
    const EnvLds e = env_lds(drl::lay::glstride(p->side), L.cells, p->n_drones, obs_k, L.obs_window, L.step_group_lanes);
    a.np = env_np(p->n_drones);
    a.lds_bm = e.bm;
    a.lds_paint = e.paint;
    a.lds_chg = e.chg;
    a.nchg = e.nchg;
    a.obs_k = obs_k;
    a.wave_lds = wave_lds_bytes(64 / L.step_group_lanes, e, obs_k > 0);
    {
        const char* v = getenv("DRL_OBS_WIDE");
        a.obs_wide = v ? atoi(v) : 1;
        const char* sp = getenv("DRL_SPECIALIZE");
        a.specialize = sp ? atoi(sp) : 1;
    }
    a.max_rounds = 1u << 20;
    a.div_side = drl::make_fastdiv((uint32_t)p->side);
    return a;
}

// dones as dwords (drl_step's write-back): whole dwords per env and per step,
// and room for an env's flags in its (dead) LDS occupancy bitmap
int dones_packed(const drl_params* p, const uint8_t* d_dones, int64_t step_stride, const drl::StepArgs& a) {
    return p->n_drones % 4 == 0 && (uintptr_t)d_dones % 4 == 0 && step_stride % 4 == 0 && a.lds_bm >= p->n_drones;
}

int launch_refill(const drl_params* p, const drl_state* s, hipStream_t stream) {
    drl::RefillArgs a;
    a.side = p->side;
    a.kbits = bit_length((uint32_t)p->side);
    a.E = s->num_envs;
    a.mt = s->mt;
    a.mt_index = s->mt_index;
    const char* lv = getenv("DRL_REFILL_LIST");  // 0: the wave-per-env kernel (A/B)
    a.list = lv ? atoi(lv) != 0 : 1;
    hipError_t e = drl::launch_refill(a, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_refill launch");
}

}  // namespace

extern "C" {

// error text for dronerl_env.cpp (hidden: not part of the ABI)
__attribute__((visibility("hidden"))) int drl_internal_fail(const char* msg) { return fail("%s", msg); }

int32_t drl_abi_version(void) { return DRL_ABI_VERSION; }

const char* drl_last_error(void) { return g_err.c_str(); }

int32_t drl_side_from_density(int32_t n_drones, double drone_density) {
    if (!(drone_density > 0.0)) return -1;
    return (int32_t)ceil(sqrt((double)n_drones / drone_density));
}

int drl_layout_query(const drl_params* p, drl_layout* out) {
    if (!out) return fail("layout is NULL");
    return validate(p, out);
}

int drl_reset(const drl_params* p, const drl_state* s, int32_t reseed, uint64_t seed_base, const uint8_t* d_env_mask,
              hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    drl::ResetArgs a;
    memset(&a, 0, sizeof a);
    const int N = p->n_drones, GG = L.cells;
    a.side = p->side;
    a.n_drones = N;
    a.cells = GG;
    a.gstride = L.ground_stride;
    a.n_sky = p->skyscrapers_factor * N;
    a.n_pack = p->packets_factor * N;
    a.n_drop = p->dropzones_factor * N;
    a.n_stat = p->stations_factor * N;
    a.E = s->num_envs;
    a.ground = s->ground;
    a.drones = s->drones;
    a.mt = s->mt;
    a.mt_index = s->mt_index;
    a.reseed = reseed ? 1 : 0;
    a.seed_base = seed_base;
    a.mask = d_env_mask;
    // Random.sample branch (random.py:496-504): pool when n <= setsize
    const int n = GG - a.n_sky;
    int setsize = 21;
    if (N > 5) setsize += (int)pow(4.0, ceil(log((double)(N * 3)) / log(4.0)));
    a.pool_branch = n <= setsize ? 1 : 0;
    a.list_cap = (GG + 7) / 8 * 8;
    a.lane_lds = (2 * a.list_cap + 128 + (a.pool_branch ? 2 * a.list_cap : 0) + 15) / 16 * 16;
    int lanes = kResetLdsTarget / a.lane_lds;
    if (lanes < 1) lanes = kLdsMax / a.lane_lds;
    if (lanes < 1) return fail("side %d: reset list does not fit LDS", p->side);
    a.lanes = lanes > 64 ? 64 : lanes;
    a.block_lds = a.lanes * a.lane_lds;
    // one wavefront per env (DRL_RESET_WAVE=0 selects the lane-per-env kernel, for A/B)
    a.wave_lds = (2 * a.list_cap + 256 + (a.pool_branch ? 2 * a.list_cap : 0) + 15) / 16 * 16;  // + the tables, below
    {
        const char* w = getenv("DRL_RESET_WAVE");
        a.wave_per_env = w ? atoi(w) : 1;
        const char* f = getenv("DRL_FY_BATCH_MIN");
        a.fy_batch_min = f ? atoi(f) : kFyBatchMin;
        if (a.fy_batch_min < 1) a.fy_batch_min = 1;
        const char* c = getenv("DRL_FY_SERIAL");
        a.fy_serial = c ? atoi(c) : kFySerial;
        a.fy_bwords = drl::lay::fy_bitmap_words(GG);
        a.wave_lds += (a.fy_bwords + 64) * 4;
        const char* wp = getenv("DRL_RESET_WPB");  // A/B knob: envs per workgroup of the wave kernel
        const int wv = wp ? atoi(wp) : 0;
        a.wpb = (wv == 1 || wv == 2 || wv == 4 || wv == 8) ? wv : 0;
        const char* pad = getenv("DRL_RESET_LDS_PAD");  // diagnostic: fewer waves per CU
        if (pad) a.wave_lds += atoi(pad) / 16 * 16;
    }
    a.div_side = drl::make_fastdiv((uint32_t)p->side);
    hipError_t e = drl::launch_reset(a, stream);
    if (e != hipSuccess) return hip_fail(e, "drl_reset launch");
    return launch_refill(p, s, stream);
}

int drl_refill(const drl_params* p, const drl_state* s, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    return launch_refill(p, s, stream);
}

int drl_mt_get(const drl_params* p, const drl_state* s, uint32_t* d_words, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_words) return fail("words is NULL");
    hipError_t e = drl::launch_mt_get(s->mt, s->mt_index, s->num_envs, d_words, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_mt_get launch");
}

int drl_mt_set(const drl_params* p, const drl_state* s, const uint32_t* d_words, int32_t* d_err, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_words) return fail("words is NULL");
    hipError_t e = drl::launch_mt_set(s->mt, s->mt_index, s->num_envs, d_words, d_err, stream);
    if (e != hipSuccess) return hip_fail(e, "drl_mt_set launch");
    return launch_refill(p, s, stream);
}

int drl_step(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards, uint8_t* d_dones,
             float* d_obs, int32_t obs_k, int32_t* d_err, hipStream_t stream) {
    return drl_step_ex(p, s, d_actions, d_rewards, d_dones, d_obs, obs_k, d_err, 0u, stream);
}

int drl_step_ex(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                uint8_t* d_dones, float* d_obs, int32_t obs_k, int32_t* d_err, uint32_t flags,
                hipStream_t stream) {
    return drl_step_code(p, s, d_actions, d_rewards, d_dones, d_obs, obs_k, nullptr, d_err, flags, stream);
}

// The policy code output of a step / obs launch: the wave's code rows are
// staged in LDS (write_obs_wave<CODE>) -- in the scratch area, which holds
// nothing else by then, when no f32 observation needs its transpose stage
// there (no extra LDS: the C3 step keeps its 32 waves per CU), else after the
// wave's LDS.
static int set_code(const drl_params* p, drl::StepArgs* a, void* d_code, const drl_layout& L, bool with_obs) {
    if ((uintptr_t)d_code % 16) return fail("code must be 16-byte aligned");
    a->code = static_cast<uint4*>(d_code);
    const int P = L.step_group_lanes, gpw = 64 / P;
    const int need = gpw * drl::lay::code_bytes(L.obs_window);
    const int stage = gpw * env_lds(drl::lay::glstride(p->side), L.cells, p->n_drones, 1, L.obs_window, P).fixed;
    if (!with_obs && stage % 16 == 0 && a->wave_lds - stage >= need) {
        a->code_lds = stage;
    } else {
        a->code_lds = (a->wave_lds + 15) / 16 * 16;  // (16-B LDS reads and writes)
        a->wave_lds = a->code_lds + need;
    }
    if (a->wave_lds > kLdsMax) return fail("the policy code needs %d B of LDS per wave", a->wave_lds);
    return 0;
}

int32_t drl_policy_code_bytes(int32_t window_radius) {
    if (window_radius < 1 || window_radius > DRL_MAX_RADIUS) return -1;
    return drl::lay::code_bytes(2 * window_radius + 1);
}

static int step_code_impl(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                          uint8_t* d_dones, float* d_obs, int32_t obs_k, void* d_code, int32_t* d_err, uint32_t flags,
                          hipStream_t stream, const drl::StepArgs* ring);

int drl_step_code(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                  uint8_t* d_dones, float* d_obs, int32_t obs_k, void* d_code, int32_t* d_err, uint32_t flags,
                  hipStream_t stream) {
    return step_code_impl(p, s, d_actions, d_rewards, d_dones, d_obs, obs_k, d_code, d_err, flags, stream, nullptr);
}

static int step_code_replay_impl(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                                 uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r,
                                 int64_t cursor, int32_t* d_err, uint32_t flags, hipStream_t stream, int synth,
                                 uint64_t synth_seed, uint64_t synth_step, int64_t env_offset);

int drl_step_code_replay(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                         uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r, int64_t cursor,
                         int32_t* d_err, uint32_t flags, hipStream_t stream) {
    return step_code_replay_impl(p, s, d_actions, d_rewards, d_dones, d_code, d_code_prev, r, cursor, d_err, flags,
                                 stream, 0, 0, 0, 0);
}

int drl_step_code_replay_synth(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                               uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r,
                               int64_t cursor, uint64_t synth_seed, uint64_t synth_step, int64_t env_offset,
                               int32_t* d_err, uint32_t flags, hipStream_t stream) {
    if (env_offset < 0) return fail("env_offset must be >= 0");
    return step_code_replay_impl(p, s, d_actions, d_rewards, d_dones, d_code, d_code_prev, r, cursor, d_err, flags,
                                 stream, 1, synth_seed, synth_step, env_offset);
}

static int step_code_replay_impl(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                                 uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r,
                                 int64_t cursor, int32_t* d_err, uint32_t flags, hipStream_t stream, int synth,
                                 uint64_t synth_seed, uint64_t synth_step, int64_t env_offset) {
    if (!d_code || !d_code_prev) return fail("code and code_prev must be non-NULL");
    if (d_code == d_code_prev) return fail("code_prev must be another buffer than code (the act's input rows)");
    if ((uintptr_t)d_code_prev % 16) return fail("code_prev must be 16-byte aligned");
    if (!r) return fail("replay is NULL");
    if (!r->obs || !r->next_obs || !r->actions || !r->rewards || !r->dones) return fail("replay buffers are NULL");
    if ((uintptr_t)r->obs % 16 || (uintptr_t)r->next_obs % 16) return fail("replay rows must be 16-byte aligned");
    if (r->capacity < 1 || cursor < 0) return fail("replay capacity must be >= 1 and cursor >= 0");
    if (!p) return fail("params is NULL");
    const int32_t cb = drl_policy_code_bytes(p->window_radius);
    if (cb < 0 || r->obs_floats * 4 != cb)
        return fail("replay obs_floats %d must hold one policy code row (%d bytes)", r->obs_floats, cb);
    drl::StepArgs ring;
    memset(&ring, 0, sizeof ring);
    const int64_t n = s ? s->num_envs : 0;
    ring.ring_first = n > r->capacity ? n - r->capacity : 0;  // as drl_replay_add: earlier rows would be overwritten
    ring.ring_cap = r->capacity;
    ring.ring_base = (cursor % r->capacity + ring.ring_first % r->capacity) % r->capacity;
    ring.ring_obs = reinterpret_cast<uint4*>(r->obs);
    ring.ring_next = reinterpret_cast<uint4*>(r->next_obs);
    ring.ring_act = r->actions;
    ring.ring_rew = r->rewards;
    ring.ring_done = r->dones;
    ring.code_prev = static_cast<const uint4*>(d_code_prev);
    ring.synth = synth;
    ring.synth_seed = synth_seed;
    ring.synth_step = synth_step;
    ring.env_offset = env_offset;
    return step_code_impl(p, s, d_actions, d_rewards, d_dones, nullptr, 0, d_code, d_err, flags, stream, &ring);
}

static int step_code_impl(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                          uint8_t* d_dones, float* d_obs, int32_t obs_k, void* d_code, int32_t* d_err, uint32_t flags,
                          hipStream_t stream, const drl::StepArgs* ring) {
    drl_layout L;
    if (flags & ~(DRL_STEP_OBS_STREAM | DRL_STEP_REFILL)) return fail("unknown drl_step flags 0x%x", flags);
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_actions || !d_rewards || !d_dones) return fail("actions/rewards/dones must be non-NULL");
    if (d_obs && (obs_k < 1 || obs_k > p->n_drones)) return fail("obs_k %d outside [1, n_drones]", obs_k);
    if (d_obs && ((uintptr_t)d_obs % 16)) return fail("obs must be 16-byte aligned");
    // (d_obs NULL with d_code: the code alone, drone index 0's window geometry)
    const int k = d_obs ? obs_k : (d_code ? 1 : 0);
    drl::StepArgs a = step_args(p, s, L, k);
    if (a.wave_lds > kLdsMax) return fail("obs_k %d needs %d B of LDS per wave", obs_k, a.wave_lds);
    a.actions = d_actions;
    a.rewards = d_rewards;
    a.dones = d_dones;
    a.obs = d_obs;
    a.err = d_err;
    a.og = obs_geom(p, L, k ? k : 1);
    a.obs_nt = (flags & DRL_STEP_OBS_STREAM) ? 1 : 0;
    a.dones_packed = dones_packed(p, d_dones, 0, a);
    if (d_code && set_code(p, &a, d_code, L, d_obs != nullptr)) return -1;
    if (ring) {
        a.ring_obs = ring->ring_obs;
        a.ring_next = ring->ring_next;
        a.ring_act = ring->ring_act;
        a.ring_rew = ring->ring_rew;
        a.ring_done = ring->ring_done;
        a.code_prev = ring->code_prev;
        a.ring_first = ring->ring_first;
        a.ring_base = ring->ring_base;
        a.ring_cap = ring->ring_cap;
        a.synth = ring->synth;
        a.env_offset = ring->env_offset;
        a.synth_seed = ring->synth_seed;
        a.synth_step = ring->synth_step;
    }
    hipError_t e = drl::launch_step(a, L.step_group_lanes, stream, drl::kStepMode);
    if (e != hipSuccess) return hip_fail(e, "drl_step launch");
    return (flags & DRL_STEP_REFILL) ? launch_refill(p, s, stream) : 0;
}

int drl_rollout(const drl_params* p, const drl_state* s, int32_t num_steps, const int32_t* d_actions,
                int64_t act_step_stride, float* d_rewards, uint8_t* d_dones, int64_t out_step_stride, float* d_obs,
                int32_t obs_k, int64_t obs_step_stride, int32_t* d_err, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (num_steps < 0) return fail("num_steps < 0");
    if (s->num_envs == 0 || num_steps == 0) return 0;
    if (!d_actions || !d_rewards || !d_dones) return fail("actions/rewards/dones must be non-NULL");
    const int64_t EN = s->num_envs * (int64_t)p->n_drones;
    if (num_steps > 1 && act_step_stride < EN) return fail("act_step_stride must be >= num_envs * n_drones");
    if (out_step_stride != 0 && out_step_stride < EN) return fail("out_step_stride must be 0 or >= num_envs * n_drones");
    if (d_obs) {
        if (obs_k < 1 || obs_k > p->n_drones) return fail("obs_k %d outside [1, n_drones]", obs_k);
        // the base 16-B aligned like drl_step; later steps' bases are 8-B aligned (strides are multiples of 6
        // floats), which the observation writer handles (16-B stores where a wave's base allows them)
        if ((uintptr_t)d_obs % 16 || obs_step_stride % 2) return fail("obs must be 16-byte aligned, obs_step_stride even");
        const int64_t per = s->num_envs * (int64_t)obs_k * L.obs_floats;
        if (obs_step_stride != 0 && obs_step_stride < per) return fail("obs_step_stride must be 0 or >= one step's obs");
    }
    drl::StepArgs a = step_args(p, s, L, d_obs ? obs_k : 0);
    if (a.wave_lds > kLdsMax) return fail("obs_k %d needs %d B of LDS per wave", obs_k, a.wave_lds);
    a.actions = d_actions;
    a.rewards = d_rewards;
    a.dones = d_dones;
    a.obs = d_obs;
    a.err = d_err;
    a.og = obs_geom(p, L, d_obs ? obs_k : 1);
    a.act_tstride = act_step_stride;
    a.out_tstride = out_step_stride;
    a.obs_tstride = d_obs ? obs_step_stride : 0;
    a.dones_packed = dones_packed(p, d_dones, out_step_stride, a);
    if (L.step_group_lanes < (d_obs ? drl::kRolloutMinLanes : drl::kRolloutNoObsMinLanes)) {
        // narrow groups (the 64-VGPR kernels): one drl_step launch per step,
        // streaming observation stores, a refill every refill_every steps
        a.obs_nt = 1;
        for (int32_t t = 0; t < num_steps; ++t) {
            a.actions = d_actions + t * act_step_stride;
            a.rewards = d_rewards + t * out_step_stride;
            a.dones = d_dones + t * out_step_stride;
            a.obs = d_obs ? d_obs + t * a.obs_tstride : nullptr;
            hipError_t e = drl::launch_step(a, L.step_group_lanes, stream, drl::kStepMode);
            if (e != hipSuccess) return hip_fail(e, "drl_rollout step launch");
            if (((t + 1) % L.refill_every == 0 || t + 1 == num_steps) && launch_refill(p, s, stream)) return -1;
        }
        return 0;
    }
    // one launch with the state on chip: the steps take respawn candidates
    // from the rings while they last and then draw from the stream (each
    // env's stream position travels with its entries); one refill at the end.
    // (Launches of refill_every steps with a refill between them were slower:
    // C5 141.8 vs 119.5 us/step, C4 30.4 vs 29.8 -- each relaunch re-stages
    // the grounds and drains the waves.)
    a.steps = num_steps;
    hipError_t e = drl::launch_step(a, L.step_group_lanes, stream, drl::kRolloutMode);
    if (e != hipSuccess) return hip_fail(e, "drl_rollout launch");
    if (launch_refill(p, s, stream)) return -1;
    return 0;
}

int drl_obs(const drl_params* p, const drl_state* s, int32_t k, float* d_obs, hipStream_t stream) {
    return drl_obs_code(p, s, k, d_obs, nullptr, stream);
}

int drl_obs_code(const drl_params* p, const drl_state* s, int32_t k, float* d_obs, void* d_code, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_obs && !d_code) return fail("obs is NULL");
    if (!d_obs) k = 1;  // the code alone: drone index 0's window
    if (k < 1 || k > p->n_drones) return fail("k %d outside [1, n_drones]", k);
    if ((uintptr_t)d_obs % 16) return fail("obs must be 16-byte aligned");
    drl::StepArgs a = step_args(p, s, L, k);
    if (a.wave_lds > kLdsMax) return fail("k %d needs %d B of LDS per wave", k, a.wave_lds);
    a.obs = d_obs;
    a.og = obs_geom(p, L, k);
    if (d_code && set_code(p, &a, d_code, L, d_obs != nullptr)) return -1;
    hipError_t e = drl::launch_step(a, L.step_group_lanes, stream, drl::kObsMode);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_obs launch");
}

int drl_decode(const drl_params* p, const drl_state* s, int32_t* d_order, int32_t* d_y, int32_t* d_x,
               int32_t* d_charge, uint8_t* d_carry, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    hipError_t e = drl::launch_decode(s->drones, s->num_envs, p->n_drones, d_order, d_y, d_x, d_charge, d_carry, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_decode launch");
}

int drl_grid_obs(const drl_params* p, const drl_state* s, float* d_grid, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_grid) return fail("grid is NULL");
    if ((uintptr_t)d_grid % 8) return fail("grid must be 8-byte aligned");
    hipError_t e = drl::launch_grid_obs(s->ground, s->drones, s->num_envs, p->side, p->n_drones, L.ground_stride, d_grid,
                                        stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_grid_obs launch");
}

int drl_code_decode(int32_t window_radius, const void* d_code, int64_t n, float* d_obs, hipStream_t stream) {
    if (window_radius < 1 || window_radius > DRL_MAX_RADIUS) return fail("window_radius outside [1, %d]", DRL_MAX_RADIUS);
    if (n < 0) return fail("n < 0");
    if (n == 0) return 0;
    if (!d_code || !d_obs) return fail("code / obs is NULL");
    if ((uintptr_t)d_code % 2 || (uintptr_t)d_obs % 8) return fail("code must be 2-byte and obs 8-byte aligned");
    hipError_t e = drl::launch_code_decode(d_code, n, 2 * window_radius + 1, d_obs, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_code_decode launch");
}

int drl_hbm_probe(const void* d_src, void* d_dst, int64_t bytes, int32_t mode, hipStream_t stream) {
    if (mode != 0 && mode != 1) return fail("mode must be 0 (copy) or 1 (read)");
    if (bytes <= 0 || bytes % 16) return fail("bytes must be a positive multiple of 16");
    if (!d_src || !d_dst) return fail("src / dst is NULL");
    if ((uintptr_t)d_src % 16 || (uintptr_t)d_dst % 16) return fail("src and dst must be 16-byte aligned");
    if (bytes / 16 >= ((int64_t)1 << 40)) return fail("bytes too large");
    hipError_t e = drl::launch_hbm_probe(d_src, d_dst, bytes, mode, 0, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_hbm_probe launch");
}

int drl_encode(const drl_params* p, const drl_state* s, const int32_t* d_order, const int32_t* d_y, const int32_t* d_x,
               const int32_t* d_charge, const uint8_t* d_carry, hipStream_t stream) {
    drl_layout L;
    if (validate(p, &L) || check_state(s, L)) return -1;
    if (s->num_envs == 0) return 0;
    if (!d_order || !d_y || !d_x || !d_charge || !d_carry) return fail("encode inputs must be non-NULL");
    hipError_t e = drl::launch_encode(s->drones, s->num_envs, p->n_drones, d_order, d_y, d_x, d_charge, d_carry, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_encode launch");
}

int drl_synth_actions(uint64_t seed, uint64_t step, int64_t env_offset, int64_t num_envs, int32_t n_drones,
                      int32_t* d_actions, hipStream_t stream) {
    if (num_envs < 0 || n_drones < 1) return fail("bad sizes");
    if (num_envs == 0) return 0;
    if (!d_actions) return fail("actions is NULL");
    hipError_t e = drl::launch_synth(seed, step, env_offset, num_envs, n_drones, d_actions, stream);
    return e == hipSuccess ? 0 : hip_fail(e, "drl_synth_actions launch");
}

}  // extern "C"
