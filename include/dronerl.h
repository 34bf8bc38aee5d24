/*
 * dronerl.h — C ABI of the MI355X-native batched DroneRL environment
 * (libdronerl.so, hand-written HIP kernels for gfx950).
 *
 * The reference (nyx-ai/droneRL) is pure Python and has no FFI; this ABI is
 * what a Python (ctypes) or any other FFI binds to replace its env hot path:
 *
 *   reference                                            this ABI
 *   torch_impl/env/env.py:68-101   DeliveryDrones.reset   drl_reset
 *   torch_impl/env/env.py:112-215  DeliveryDrones.step    drl_step
 *   torch_impl/env/wrappers.py:55-73 WindowedGridView     drl_obs (or drl_step's fused obs)
 *   torch_impl/env/wrappers.py:34-43 GridView             drl_grid_obs
 *   jax_impl/env/env.py:89-135     DeliveryDrones.reset   drl_reset (batched over envs)
 *   jax_impl/env/env.py:137-250    DeliveryDrones.step    drl_step  (batched over envs)
 *   jax_impl/env/env.py:274-309    DeliveryDrones.get_obs drl_obs
 *   jax_impl/env/env.py:11-35      DroneEnvParams/State   drl_params / drl_state + drl_decode
 *   torch_impl/helpers/rl_helpers.py:12-18 set_seed       drl_reset(reseed=1)
 *   jax_impl/agents/dqn.py:132-146 DQNAgent.act          drl_qnet_act* (drl_qnet_act_eps: epsilon on device)
 *   jax_impl/agents/dqn.py:147-200 train_step / update_target / update_epsilon,
 *   jax_impl/buffers.py:79-93      sample / can_sample,
 *   train_jax.py:68-98             the scan body's learner block   drl_dqn_train
 *   jax_impl/buffers.py:57-77      ReplayBuffer.add_many  drl_replay_add
 *   train_jax.py:55-62             env.step + add_many    drl_step_code_replay (one launch)
 *   train_jax.py:42-62             + the random drones    drl_step_code_replay_synth (drawn in the step)
 *
 * Two layers: stateless calls on caller-owned buffers (drl_reset, drl_step,
 * ...) and library-owned env handles (drl_env_*) that
 * forward to them.
 *
 * Semantics are torch_impl's, bit-exact (state, dict order, done flags, RNG
 * stream), with each env carrying its own CPython-compatible MT19937 stream:
 * env e behaves exactly like `random.seed(seed_base + e); env.reset()` followed
 * by env.step(...) calls in the reference.
 *
 * Conventions
 *  - All data pointers are DEVICE pointers on the current HIP device.
 *  - The caller owns every buffer (state included: size them with
 *    drl_layout_query).  No call allocates, frees or synchronises, so every
 *    call is hipGraph-capturable; all work is enqueued on `stream`.
 *  - Return 0 on success, <0 on error (text: drl_last_error(), thread-local).
 *  - Actions/rewards/dones are indexed by drone index [E][n_drones]; the
 *    state's drone records are kept in dict order (the reference's hidden
 *    iteration order O, env.py:124).
 */
#ifndef DRONERL_H
#define DRONERL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

#define DRL_ABI_VERSION 9
/* Per-env RNG row of `mt` (u32 words, 7104 B):
 *   [0, 624)     MT19937 block 0     the env's CPython stream lives in block
 *   [624, 1248)  MT19937 block 1     mt_index.par; the other block holds the
 *                                    next block (twisted by drl_refill) or scratch
 *   [1248, 1760) respawn-candidate ring (DRL_CAND_SLOTS entries, see drl_refill)
 *   1760         the stream position just after the ring's last entry: MT
 *                index | block << 10 (valid while the ring holds entries)
 *   [1761, 1776) padding (rows 64-B aligned) */
#define DRL_MT_WORDS 1776
#define DRL_MT_BLOCK1 624
#define DRL_MT_RING 1248
#define DRL_MT_RING_END 1760
#define DRL_CAND_SLOTS 512
#define DRL_MAX_DRONES 64
#define DRL_MAX_SIDE 128
#define DRL_MAX_RADIUS 8

/* object codes (common/constants.py:15-19) */
#define DRL_EMPTY 0
#define DRL_SKYSCRAPER 2
#define DRL_STATION 3
#define DRL_DROPZONE 4
#define DRL_PACKET 5

/* error bits written to drl_step's optional err word */
#define DRL_ERR_BAD_ACTION 1   /* action outside [-5, 4] (IndexError in the reference) */
#define DRL_ERR_NO_FREE_CELL 2 /* respawn found no free cell (the reference loops forever) */
#define DRL_ERR_BAD_STATE 4    /* drl_env_set_state: MT index outside [0, 624] (CPython setstate's ValueError;
                                  clamped to 624), or a ground code outside {0, 2, 3, 4, 5} (stored as
                                  its low 4 bits) */
#define DRL_ERR_QNET_RANGE 8   /* drl_qnet_act (DRL_QNET_F32): an input or hidden activation at or beyond fp16's
                                  range (|v| >= 65520) or NaN; that env's Q values are not valid */

/* Env parameters: torch_impl DEFAULT_CONFIG (env.py:28-42) / jax DroneEnvParams
 * (jax env.py:11-26).  `side` is explicit; torch_impl derives it as
 * ceil(sqrt(n_drones / drone_density)) (env.py:75): see drl_side_from_density. */
typedef struct drl_params {
    int32_t side;
    int32_t n_drones;
    int32_t charge;     /* >= 0 */
    int32_t discharge;  /* >= 0 */
    int32_t packets_factor;
    int32_t dropzones_factor;
    int32_t stations_factor;
    int32_t skyscrapers_factor;
    int32_t window_radius; /* 1..DRL_MAX_RADIUS */
    float pickup_reward;
    float delivery_reward;
    float crash_reward;
    float charge_reward;
} drl_params;

/* Buffer geometry for a params set. */
typedef struct drl_layout {
    int32_t side;
    int32_t n_drones;
    int32_t cells;          /* side*side */
    int32_t ground_stride;  /* bytes per env in `ground`: ceil(cells / 2) rounded up to 16 (packed nibbles) */
    int32_t drone_stride;   /* u32 records per env in `drones` (== n_drones) */
    int32_t mt_stride;      /* u32 words per env in `mt` (== DRL_MT_WORDS) */
    int32_t obs_window;     /* 2*radius+1 */
    int32_t obs_floats;     /* floats per observed drone: window^2 * 6 */
    int32_t step_group_lanes; /* wavefront lanes per env in drl_step */
    int32_t step_lds_bytes;   /* dynamic LDS per block (one wavefront) of drl_step */
    int32_t cand_slots;       /* respawn-candidate ring entries per env (DRL_CAND_SLOTS) */
    int32_t refill_every;     /* recommended drl_refill cadence in steps (DRL_STEP_REFILL) */
} drl_layout;

/* Device state of num_envs envs (structure of arrays, env-major).
 *  ground : u8  [E][ground_stride]  object code per cell (row-major k = y*side+x), packed
 *           two cells per byte (ABI 8): cell k in bits 4*(k&1)..+3 of byte k/2
 *           (the codes are < 8; half the HBM bytes of a byte per cell; the
 *           kernels unpack into LDS).  drl_env_get_state / set_state and
 *           BatchedDeliveryDrones.decode / set_state convert to a byte per cell.
 *  drones : u32 [E][n_drones]       one record per drone in dict order:
 *           bits 0-7 y, 8-15 x, 16-23 charge, 24 carrying, 25-31 drone index
 *  mt     : u32 [E][DRL_MT_WORDS]   two MT19937 blocks + the candidate ring (above)
 *  mt_index: u32 [E]                bits 0-9 CPython's MT index (next word; 624 =
 *                                   twist first), bit 10 `par` (the block holding
 *                                   the stream), bits 11-19 ring head, bits 20-29
 *                                   ring count; kept apart so a wave's envs share
 *                                   one cache line.  A plain CPython index (0..624,
 *                                   upper bits 0) is a valid word: block 0, empty ring.
 *
 * The candidate ring is a cache of the env's FUTURE respawn cells: entry k is
 * the k-th (y, x) pair of accepted randint(0, side-1) draws ahead of the
 * stream position (bits 0-13 cell y*side+x, bits 16-25 the MT index after its
 * second draw, bit 26 that index's block).  Those cells depend on the stream
 * alone, not on the board, so drl_refill can draw them in bulk off the step's
 * critical path; drl_step consumes them in order, rejects occupied ones
 * exactly as env.py:226-233 does, and falls back to drawing from the stream
 * itself when the ring runs dry.  Results never depend on the ring's fill
 * level: it only moves MT work out of the step. */
typedef struct drl_state {
    uint8_t* ground;
    uint32_t* drones;
    uint32_t* mt;
    uint32_t* mt_index;
    int64_t num_envs;
} drl_state;

int32_t drl_abi_version(void);
const char* drl_last_error(void);

/* ceil(sqrt(n_drones / drone_density)) in double, as env.py:75 computes it. */
int32_t drl_side_from_density(int32_t n_drones, double drone_density);

/* Validate params and fill the layout.  Errors mirror the reference's
 * ValueErrors (spawn_objects env.py:59-60, sample, jax env.py:96-104). */
int drl_layout_query(const drl_params* p, drl_layout* out);

/* reset() for every env (or every env with d_env_mask[e] != 0).
 * reseed != 0: first re-seed env e's stream as random.seed(seed_base + e)
 * (rl_helpers.py:18), then draw the reset exactly like env.py:68-101.
 * reseed == 0: continue each env's current stream (a plain env.reset()).
 * Ends with a drl_refill of the respawn-candidate rings. */
int drl_reset(const drl_params* p, const drl_state* s, int32_t reseed, uint64_t seed_base,
              const uint8_t* d_env_mask, hipStream_t stream);

/* step(actions) for every env (env.py:112-215).  d_actions int32 [E][n_drones]
 * by drone index; d_rewards f32 [E][n_drones]; d_dones u8 [E][n_drones].
 * d_obs (nullable): fused WindowedGridView observation of drone indices
 * 0..obs_k-1 after the step, f32 [E][obs_k][W][W][6].
 * d_err (nullable): OR-ed DRL_ERR_* bits. */
int drl_step(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
             uint8_t* d_dones, float* d_obs, int32_t obs_k, int32_t* d_err, hipStream_t stream);

/* drl_step with flags (drl_step == drl_step_ex with flags 0).
 * DRL_STEP_OBS_STREAM: write the observation with streaming (non-temporal)
 * stores, for observations no kernel reads right away (rollout output).
 * Without it the stores are cached, so a consumer launched next (the policy's
 * act) reads them from the caches.  Results are identical either way. */
#define DRL_STEP_OBS_STREAM 1u
/* DRL_STEP_REFILL: launch drl_refill after the step (callers pass it every
 * layout.refill_every steps; the Python env and the env handles do). */
#define DRL_STEP_REFILL 2u
int drl_step_ex(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                uint8_t* d_dones, float* d_obs, int32_t obs_k, int32_t* d_err, uint32_t flags,
                hipStream_t stream);

/* num_steps steps (jax_impl run_steps, env/env.py:252-272, with the rewards,
 * dones and observation of every step): identical results to num_steps
 * drl_step calls.  Step t reads d_actions + t * act_step_stride and writes
 * d_rewards / d_dones + t * out_step_stride and d_obs + t * obs_step_stride
 * (element strides; out/obs stride 0 = every step overwrites the same
 * buffer, leaving the last step's).  With layout.step_group_lanes >= 16 the
 * steps run in one launch with the state on chip, written back once at the
 * end (respawns take ring entries while they last, then draw from the
 * stream); narrower groups run one drl_step launch per step with a refill
 * every layout.refill_every steps.  Ends with a drl_refill either way. */
int drl_rollout(const drl_params* p, const drl_state* s, int32_t num_steps, const int32_t* d_actions,
                int64_t act_step_stride, float* d_rewards, uint8_t* d_dones, int64_t out_step_stride, float* d_obs,
                int32_t obs_k, int64_t obs_step_stride, int32_t* d_err, hipStream_t stream);

/* Extend every env's respawn-candidate ring (see drl_state) through the end
 * of the MT block after the stream's: an env whose ring does not reach past
 * the stream's block gets the rest of that block's draws and, twisted into
 * the other block's words, all of the next block's (up to DRL_CAND_SLOTS
 * entries).  Never changes the env's observable state.  drl_reset and
 * drl_mt_set end with one. */
int drl_refill(const drl_params* p, const drl_state* s, hipStream_t stream);

/* The envs' CPython getstate() words: d_words u32 [E][625] = the 624 state
 * words of the stream's block + the MT index (what random.getstate() holds). */
int drl_mt_get(const drl_params* p, const drl_state* s, uint32_t* d_words, hipStream_t stream);
/* random.setstate() for every env from d_words u32 [E][625] (then a refill).
 * An index outside [0, 624] is clamped to 624 and raises DRL_ERR_BAD_STATE in
 * d_err (nullable). */
int drl_mt_set(const drl_params* p, const drl_state* s, const uint32_t* d_words, int32_t* d_err, hipStream_t stream);

/* WindowedGridView observation (wrappers.py:10-31,55-73) of drone indices
 * 0..k-1: f32 [E][k][W][W][6]. */
int drl_obs(const drl_params* p, const drl_state* s, int32_t k, float* d_obs, hipStream_t stream);

/* Policy code (ABI 7): drone index 0's window as one u16 per cell -- object
 * code (bits 0-2, walls as DRL_SKYSCRAPER) | ((charge+1) | carry << 7) << 3
 * (0 above: no drone) -- in four groups of ceil(W*W/4) cells, each padded
 * with zero codes to a multiple of 8.  Bytes per env (16-B multiple): */
int32_t drl_policy_code_bytes(int32_t window_radius);
/* drl_step_ex that also writes the policy code of the state after the step
 * (d_code, 16-B aligned, [E][drl_policy_code_bytes]): what drl_qnet_act_code
 * reads instead of the observation.  With d_obs non-NULL the observation
 * (obs_k >= 1) is written as well; with d_obs NULL the code alone (obs_k
 * ignored): a consumer that only needs drone 0's window skips the f32 rows
 * (6 floats per cell) entirely.  d_code NULL: exactly drl_step_ex. */
int drl_step_code(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                  uint8_t* d_dones, float* d_obs, int32_t obs_k, void* d_code, int32_t* d_err, uint32_t flags,
                  hipStream_t stream);
/* Policy code rows -> drone index 0's observation, f32 [n][W][W][6] exactly
 * as drl_obs writes it (a replay buffer of codes decodes its samples). */
int drl_code_decode(int32_t window_radius, const void* d_code, int64_t n, float* d_obs, hipStream_t stream);
/* Measurement helper (the measured copy-kernel peak beside
 * the spec): mode 0 copies `bytes` from d_src to d_dst, mode 1 only reads
 * d_src (d_dst, at least `bytes` long, may be written).  A plain float4
 * copy: one 16-B element per lane, a grid over the buffer.  Time it with
 * events on `stream`. */
int drl_hbm_probe(const void* d_src, void* d_dst, int64_t bytes, int32_t mode, hipStream_t stream);
/* drl_obs that also writes the policy code (d_code nullable); d_obs NULL:
 * the code alone (k ignored). */
int drl_obs_code(const drl_params* p, const drl_state* s, int32_t k, float* d_obs, void* d_code, hipStream_t stream);

/* GridView observation (wrappers.py:10-31,34-43): the [side][side][6] f32
 * base grid of every env (each drone of an env sees the same grid):
 * d_grid f32 [E][side][side][6], channels as drl_obs, no wall padding. */
int drl_grid_obs(const drl_params* p, const drl_state* s, float* d_grid, hipStream_t stream);

/* Decode drone records to per-index vectors (jax DroneEnvState fields):
 * d_order[E][N] = drone index at dict position; y/x/charge/carry [E][N] by
 * drone index.  Any output may be NULL. */
int drl_decode(const drl_params* p, const drl_state* s, int32_t* d_order, int32_t* d_y, int32_t* d_x,
               int32_t* d_charge, uint8_t* d_carry, hipStream_t stream);

/* Inverse of drl_decode (hand-built states, as jax_tests/test_env.py:14-110 do).
 * charge must lie in [0, 100]. */
int drl_encode(const drl_params* p, const drl_state* s, const int32_t* d_order, const int32_t* d_y,
               const int32_t* d_x, const int32_t* d_charge, const uint8_t* d_carry, hipStream_t stream);

/* Synthetic uniform actions in {0..4} from a counter hash of
 * (seed, step, env_offset + e, drone) — identical to the oracle's stream. */
int drl_synth_actions(uint64_t seed, uint64_t step, int64_t env_offset, int64_t num_envs, int32_t n_drones,
                      int32_t* d_actions, hipStream_t stream);

/* ------------------------------------------------------------------------
 * Env handles: the library owns the state of num_envs
 * envs on one device; the caller owns actions/rewards/dones/obs.  Every call
 * except create/destroy/errors is asynchronous on `stream` and allocation-free.
 * A handle is single-threaded; use one per device/process.
 *
 *   B2 row                      here
 *   drl_create/drl_destroy      drl_env_create / drl_env_destroy
 *   drl_reset(env, mask)        drl_env_reset (set_seed: drl_env_seed)
 *   drl_step(env, ...)          drl_env_step / drl_env_step_obs (fused obs)
 *   drl_obs(env, k, obs)        drl_env_obs
 *   drl_get_state/set_state     drl_env_get_state / drl_env_set_state
 * ------------------------------------------------------------------------ */
typedef struct drl_env drl_env;

/* SoA view of an env batch (device pointers, dense, env-major):
 *  ground u8 [E][side*side]; order/y/x/charge i32 [E][n_drones] (order = drone
 *  index at dict position, the rest by drone index); carry u8 [E][n_drones];
 *  mt u32 [E][625] = CPython's getstate() words 0..623 + index. */
typedef struct drl_state_view {
    uint8_t* ground;
    int32_t* order;
    int32_t* y;
    int32_t* x;
    int32_t* charge;
    uint8_t* carry;
    uint32_t* mt;
} drl_state_view;

/* Allocate the state of num_envs envs on `device`.  Global env index of env e
 * is env_offset + e (train_jax.py:196-212 sharding); the first drl_env_reset
 * seeds env e as random.seed(base_seed + env_offset + e). */
int drl_env_create(const drl_params* p, int32_t device, int64_t num_envs, int64_t env_offset, uint64_t base_seed,
                   drl_env** out);
int drl_env_destroy(drl_env* env);
/* set_seed (rl_helpers.py:12-18): the next reset re-seeds from base_seed. */
int drl_env_seed(drl_env* env, uint64_t base_seed);
/* reset() (env.py:68-101) of every env, or of envs with d_env_mask[e] != 0
 * (the first reset after create/seed must cover every env). */
int drl_env_reset(drl_env* env, const uint8_t* d_env_mask, hipStream_t stream);
/* step() (env.py:112-215): actions i32, rewards f32, dones u8, [E][n_drones]. */
int drl_env_step(drl_env* env, const int32_t* d_actions, float* d_rewards, uint8_t* d_dones, hipStream_t stream);
/* step() + the WindowedGridView observation of drone indices 0..k-1 after it
 * (cached stores at layout.step_group_lanes 8 or less, streaming stores at 16
 * and more: the faster mode when the policy reads the observation next). */
int drl_env_step_obs(drl_env* env, const int32_t* d_actions, float* d_rewards, uint8_t* d_dones, int32_t k,
                     float* d_obs, hipStream_t stream);
/* WindowedGridView observation (wrappers.py:55-73): f32 [E][k][W][W][6]. */
int drl_env_obs(drl_env* env, int32_t k, float* d_obs, hipStream_t stream);
/* GridView observation (wrappers.py:34-43): f32 [E][side][side][6]. */
int drl_env_grid_obs(drl_env* env, float* d_grid, hipStream_t stream);
/* Copy the state out to / in from a caller-owned SoA view (NULL fields are
 * skipped by get_state; set_state needs all of them and trusts their
 * validity: positions on the grid, distinct cells, charge in [0, 100]; ground
 * codes are common/constants.py Object values {0, 2, 3, 4, 5} (< 8: the
 * packed ground holds a nibble per cell, the policy code 3 bits); an MT index
 * outside [0, 624] is clamped to 624, and a ground code outside that set is
 * stored as its low 4 bits; both raise DRL_ERR_BAD_STATE in the handle's
 * error word). */
int drl_env_get_state(drl_env* env, const drl_state_view* v, hipStream_t stream);
int drl_env_set_state(drl_env* env, const drl_state_view* v, hipStream_t stream);
/* The handle's raw buffers, params and layout (any output may be NULL). */
int drl_env_state(const drl_env* env, drl_state* s, drl_params* p, drl_layout* L);
/* Synchronise `stream`, read the OR of DRL_ERR_* bits raised by steps, and
 * clear them when `clear` != 0. */
int drl_env_errors(drl_env* env, int32_t* flags, int32_t clear, hipStream_t stream);

/* ------------------------------------------------------------------------
 * DQN consumer of the observation, on MFMA: the dense Q-network of jax_impl/agents/dqn.py:47-63
 * (Dense(h) + ReLU per hidden layer, then Dense(n_actions)) and the
 * epsilon-greedy act of dqn.py:132-146 for every env (train_jax.py:42-49:
 * drone 0 follows the agent), plus ReplayBuffer.add_many (buffers.py:57-80).
 *
 * Precision (drl_qnet_desc.precision):
 *   DRL_QNET_BF16: bf16 operands, f32 accumulation (one MFMA per tile and
 *     K-slice); Q within ~1e-2 relative of the f32 forward.
 *   DRL_QNET_F32: the reference's f32 nets (jax dqn.py:47-63 / torch
 *     dqn.py:44-82 run in f32): every operand v is split exactly enough into
 *     fp16 hi = fp16(v) and lo = fp16((v - hi) * 2^11); products hi*hi go to
 *     one f32 accumulator and hi*lo + lo*hi to a second, combined as
 *     acc_hi + 2^-11 * acc_lo (the lo*lo term, <= 2^-22 relative, is
 *     dropped).  Q matches an f32 forward to f32 rounding (~1e-6 relative).
 *     Range: |weights|, |inputs| and |hidden activations| < 65504 (fp16).
 * ------------------------------------------------------------------------ */
#define DRL_QNET_BF16 0
#define DRL_QNET_F32 1
/* input: DRL_QNET_INPUT_OBS, the f32 observation rows (drl_qnet_act); or
 * DRL_QNET_INPUT_CODE, drone index 0's policy code written by drl_step_code /
 * drl_obs_code (drl_qnet_act_code; DRL_QNET_F32, window radius 2..4).  The
 * weights are the same; the packed layout differs. */
#define DRL_QNET_INPUT_OBS 0
#define DRL_QNET_INPUT_CODE 1
typedef struct drl_qnet_desc {
    int32_t in_features;  /* observation floats, W*W*6 (even, <= 512) */
    int32_t n_hidden;     /* 1..3 hidden layers */
    int32_t hidden[3];    /* widths: multiples of 32 in [32, 128] */
    int32_t n_actions;    /* 1..8 (Action.num_actions() = 5) */
    int32_t precision;    /* DRL_QNET_BF16 or DRL_QNET_F32 */
    int32_t input;        /* DRL_QNET_INPUT_OBS or DRL_QNET_INPUT_CODE (ABI 7) */
} drl_qnet_desc;

/* Bytes of the packed network (weight fragments + f32 biases; DRL_QNET_F32
 * packs fp16 hi and lo fragments: layer 0's hi and lo sets first when both
 * fit the 160 KB LDS together, else the hi fragments where bf16 ones go and
 * the lo fragments after them).  The layout is opaque to callers. */
int drl_qnet_packed_bytes(const drl_qnet_desc* d, int64_t* bytes);
/* Pack the network once per weight update.  d_weights / d_biases: host arrays
 * of n_hidden + 1 device pointers; layer l weights f32 [out][in] row-major
 * (torch nn.Linear; a flax Dense kernel is its transpose), biases f32 [out].
 * d_packed: 16-byte aligned device buffer of drl_qnet_packed_bytes. */
int drl_qnet_pack(const drl_qnet_desc* d, const float* const* d_weights, const float* const* d_biases, void* d_packed,
                  hipStream_t stream);
/* actions[e * action_stride] = u_e < epsilon ? random action : argmax_a Q(obs_e)
 * for e < num_envs (first maximum on ties, like jnp.argmax).  obs f32 rows of
 * obs_stride floats (8-byte aligned).  u_e and the random action come from a
 * counter hash of (seed, step, env_offset + e).  d_q (nullable): Q f32
 * [num_envs][n_actions].  d_err (nullable): OR-ed DRL_ERR_QNET_RANGE. */
int drl_qnet_act(const drl_qnet_desc* d, const void* d_packed, const float* d_obs, int64_t num_envs,
                 int64_t obs_stride, float epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                 int32_t* d_actions, int64_t action_stride, float* d_q, int32_t* d_err, hipStream_t stream);
/* drl_qnet_act for column 0 of d_actions [num_envs][n_drones] (contiguous
 * rows), fused with drl_synth_actions(synth_seed, synth_step, env_offset,
 * num_envs, n_drones) for columns 1..n_drones-1: one launch for the
 * train_jax.py:42-49 action row (drone 0 from the agent, the others from the
 * synthetic stream), identical to the two calls in sequence.  n_drones >= 1. */
int drl_qnet_act_synth(const drl_qnet_desc* d, const void* d_packed, const float* d_obs, int64_t num_envs,
                       int64_t obs_stride, float epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                       int32_t* d_actions, int32_t n_drones, uint64_t synth_seed, uint64_t synth_step, float* d_q,
                       int32_t* d_err, hipStream_t stream);

/* drl_qnet_act for a DRL_QNET_INPUT_CODE net, reading drone index 0's policy
 * code (d_code, drl_policy_code_bytes(radius) per env, as drl_step_code /
 * drl_obs_code write it) instead of the f32 observation: the 0/1 and
 * charge/100 inputs are computed from the code exactly as the observation
 * holds them, so Q is the f32 net's on the same window (to f32 rounding).
 * synth_n > 1: as drl_qnet_act_synth (columns 1..synth_n-1 of d_actions from
 * drl_synth_actions(synth_seed, synth_step), action_stride = synth_n). */
int drl_qnet_act_code(const drl_qnet_desc* d, const void* d_packed, const void* d_code, int64_t num_envs,
                      float epsilon, uint64_t seed, uint64_t step, int64_t env_offset, int32_t* d_actions,
                      int64_t action_stride, int32_t synth_n, uint64_t synth_seed, uint64_t synth_step, float* d_q,
                      int32_t* d_err, hipStream_t stream);

/* Replay ring buffer storage (device, caller-owned): obs/next_obs f32
 * [capacity][obs_floats], actions i32, rewards f32, dones u8 [capacity].
 * Rows are copied bit for bit: policy-code rows (drl_policy_code_bytes / 4
 * words each) store the same way. */
typedef struct drl_replay {
    int64_t capacity;
    int32_t obs_floats;
    float* obs;
    float* next_obs;
    int32_t* actions;
    float* rewards;
    uint8_t* dones;
} drl_replay;

/* add_many: transition i -> slot (cursor + i) % capacity, i < n; strides in
 * elements (e.g. action_stride = n_drones to take drone 0 of [E][n_drones]).
 * With n > capacity only the last `capacity` transitions are written (what a
 * sequential add() loop leaves).  The caller advances cursor by n. */
int drl_replay_add(const drl_replay* r, int64_t cursor, int64_t n, const float* d_obs, int64_t obs_stride,
                   const float* d_next_obs, int64_t next_obs_stride, const int32_t* d_actions, int64_t action_stride,
                   const float* d_rewards, int64_t reward_stride, const uint8_t* d_dones, int64_t done_stride,
                   hipStream_t stream);
/* drl_step_code (no f32 observation) fused with the drl_replay_add of the
 * step's drone-0 transitions, code rows (replaces train_jax.py:55-62's
 * env.step + buffer.add_many pair, jax_impl/buffers.py:57-80): env e lands
 * in slot (cursor + e) % capacity with obs = d_code_prev row e (the rows the
 * act read; another buffer than d_code), next_obs = the code this step
 * writes to d_code, action = d_actions[e * n_drones], reward / done = drone
 * index 0's.  The ring's contents equal drl_step_code + drl_replay_add(obs =
 * d_code_prev, next_obs = d_code, action/reward/done column 0) bit for bit;
 * r->obs_floats * 4 = drl_policy_code_bytes(window_radius), rows 16-byte
 * aligned.  The caller advances cursor by num_envs. */
int drl_step_code_replay(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                         uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r, int64_t cursor,
                         int32_t* d_err, uint32_t flags, hipStream_t stream);
/* drl_step_code_replay whose drone indices 1..n_drones-1 act as drl_synth_actions(synth_seed, synth_step,
 * env_offset) writes them (train_jax.py:42-49: every drone but drone 0 acts at random; the same counter hash,
 * drawn inside the step): d_actions is read at column 0 only (d_actions[e * n_drones], the agent's action), its
 * other columns are neither read nor written.  Bit for bit drl_synth_actions into d_actions' columns >= 1 +
 * drl_step_code_replay.  In the train loop it replaces drl_qnet_act_synth's columns (no 4 B per drone written
 * by the act and read back by the step). */
int drl_step_code_replay_synth(const drl_params* p, const drl_state* s, const int32_t* d_actions, float* d_rewards,
                               uint8_t* d_dones, void* d_code, const void* d_code_prev, const drl_replay* r,
                               int64_t cursor, uint64_t synth_seed, uint64_t synth_step, int64_t env_offset,
                               int32_t* d_err, uint32_t flags, hipStream_t stream);


/* drl_qnet_act / drl_qnet_act_code with epsilon read from device memory
 * (d_epsilon: e.g. the learner's drl_dqn_counters.epsilon, which drl_dqn_train
 * decays on the device), so a captured graph of the train loop acts with the
 * current schedule.  d_input: the f32 observation rows (obs_stride floats) of
 * a DRL_QNET_INPUT_OBS net, or the policy code of a DRL_QNET_INPUT_CODE net
 * (obs_stride ignored).  synth_n > 1: drl_qnet_act_synth's columns. */
int drl_qnet_act_eps(const drl_qnet_desc* d, const void* d_packed, const void* d_input, int64_t num_envs,
                     int64_t obs_stride, const float* d_epsilon, uint64_t seed, uint64_t step, int64_t env_offset,
                     int32_t* d_actions, int64_t action_stride, int32_t synth_n, uint64_t synth_seed,
                     uint64_t synth_step, float* d_q, int32_t* d_err, hipStream_t stream);

/* ------------------------------------------------------------------------
 * DQN learner (the train half): one drl_dqn_train call is the
 * learner block of one train_jax.py scan step (:68-98):
 *   if current_size >= batch (buffers.py:92-93 can_sample):
 *       batch = sample(replay) (buffers.py:79-90: uniform rows in [0, size));
 *       train_step (jax_impl/agents/dqn.py:147-183): q = Q(obs)[action],
 *       td = reward + gamma * max_a Q_target(next_obs) * (1 - done),
 *       loss = mean((q - td)^2), gradient, optax.adam(learning_rate, beta1,
 *       beta2, adam_eps) update;
 *   if step % target_update_interval == 0: target = tau * online + (1 - tau)
 *       * target (dqn.py:185-190, optax.incremental_update);
 *   if step % epsilon_decay_every == 0: epsilon = max(epsilon * decay, end)
 *       (dqn.py:192-200);
 *   step += 1.
 * The step counter, Adam count, epsilon and bias-correction powers live in the
 * agent block on the device (drl_dqn_counters), so the call is graph-capturable
 * and a replayed graph continues the schedule.  The online net's packed image
 * (drl_qnet_pack's layout, d_packed) is refreshed by the same call, ready for
 * the next act.  Row sampling: a counter hash of (sample_seed, step, row) --
 * the reference's jax.random stream is jax-only.  Numerics: f32 throughout,
 * each product and sum rounded in a fixed order (oracle/dqn_learner.py).
 * Dense nets of drl_qnet_desc (1-3 hidden layers, <= 128 wide, <= 8 actions).
 * ------------------------------------------------------------------------ */
typedef struct drl_dqn_hparams {
    int32_t batch;                  /* sample batch, 1..64 (train_jax.py --batch_size, 8) */
    int32_t target_update_interval; /* >= 1 (--target_update_interval, 10) */
    int32_t epsilon_decay_every;    /* >= 1 (--epsilon_decay_every, 5) */
    int32_t reserved;               /* 0 */
    double gamma;                   /* 0.9 (--gamma) */
    double learning_rate;           /* 1e-3 (--learning_rate) */
    double beta1, beta2, adam_eps;  /* optax.adam defaults 0.9, 0.999, 1e-8 */
    double tau;                     /* 1.0 (--tau) */
    double epsilon_decay, epsilon_end;  /* train_jax.py:133-136; --epsilon_end 0.01 */
    uint64_t sample_seed;
} drl_dqn_hparams;

/* Device counters at counters_off of the agent block. */
typedef struct drl_dqn_counters {
    int32_t step;        /* the scan step (train_jax.py carry `step`) */
    int32_t count;       /* Adam steps taken (optax ScaleByAdamState.count) */
    float epsilon;       /* the act's exploration rate */
    float loss;          /* the last train_step's loss (0 without a sample) */
    double beta1_pow, beta2_pow;  /* beta^count */
    int32_t internal[8]; /* the learner's own: arrival ticket, the step's plan */
} drl_dqn_counters;

/* The agent block (device, caller-owned, one allocation of `bytes`, 16-B
 * aligned): four parameter sets (online, target, Adam mu, Adam nu) of n_params
 * floats each -- layer l's weight [out][in] row-major (torch nn.Linear) at
 * weight_off[l], its bias at bias_off[l] (floats from the set's start) --, the
 * counters, and the learner's scratch. */
typedef struct drl_dqn_layout {
    int64_t n_params;
    int64_t weight_off[4], bias_off[4];
    int64_t online_off, target_off, m_off, v_off;  /* bytes */
    int64_t counters_off, scratch_off, bytes;       /* bytes */
    int32_t grad_workgroups, grad_lds_bytes;        /* the learner launch: workgroups, dynamic LDS (informative) */
} drl_dqn_layout;

int drl_dqn_layout_query(const drl_qnet_desc* d, int32_t batch, drl_dqn_layout* layout);
/* Zero the Adam moments, the counters (a timeout flag included) and the whole
 * scratch (the hand-off granules must start untagged, whether the block comes
 * from hipMalloc or has trained before), epsilon = epsilon_start (dqn.py:116-130:
 * optax.adam's init, epsilon_start).  The caller writes the online and target
 * parameters (the reference initialises them from different keys,
 * dqn.py:114-121).  Synchronises `stream` (a host table is uploaded). */
int drl_dqn_init(const drl_qnet_desc* d, int32_t batch, void* d_agent, float epsilon_start, hipStream_t stream);
/* One learner step on replay `r` holding `size` transitions (current_size,
 * 0 <= size <= capacity).  The replay's rows: f32 observations (obs_floats >=
 * in_features) for a DRL_QNET_INPUT_OBS net, policy code rows
 * (drl_policy_code_bytes / 4 words) for a DRL_QNET_INPUT_CODE one.  d_packed:
 * the online net's packed image (drl_qnet_pack of the online set).
 * The launch's grad_workgroups poll each other's hand-offs, so they must be
 * co-resident: the call fails (-1) on a device that cannot hold them all at
 * once (e.g. a 32-CU partition).  A workgroup that gives up on a hand-off
 * (a bounded wait) sets internal[5] of the counters; from then on every call
 * returns on the device without touching the block, until drl_dqn_init. */
int drl_dqn_train(const drl_qnet_desc* d, const drl_dqn_hparams* h, void* d_agent, void* d_packed,
                  const struct drl_replay* r, int64_t size, hipStream_t stream);
/* A drl_replay_add batch (its arguments; strides in elements, obs strides in
 * 32-bit words). */
typedef struct drl_replay_batch {
    int64_t cursor, n;
    const void* obs;
    int64_t obs_stride;
    const void* next_obs;
    int64_t next_obs_stride;
    const int32_t* actions;
    int64_t action_stride;
    const float* rewards;
    int64_t reward_stride;
    const uint8_t* dones;
    int64_t done_stride;
} drl_replay_batch;
/* drl_dqn_train as if drl_replay_add(r, fresh->cursor, fresh->n, ...) had
 * already run (`size` counts its rows): the rows that add writes are read
 * from its own buffers, so the add may run concurrently on another stream
 * (the learner reads no slot it writes). */
int drl_dqn_train_fresh(const drl_qnet_desc* d, const drl_dqn_hparams* h, void* d_agent, void* d_packed,
                        const struct drl_replay* r, int64_t size, const drl_replay_batch* fresh, hipStream_t stream);

/* The `batch` replay slots (int64, [0, size)) the next drl_dqn_train on this
 * block draws: the same counter hash of (sample_seed, step, row), with the step
 * the counters hold when this launch runs on `stream`.  A sharded caller
 * gathers those rows from the ranks that own them before the train call
 * (the global learner; jax_impl/buffers.py:79-90 sample over
 * one global ring, train_jax.py:196-212). */
int drl_dqn_sample_rows(const drl_qnet_desc* d, const drl_dqn_hparams* h, const void* d_agent, int64_t size,
                        int64_t* d_slots, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DRONERL_H */
