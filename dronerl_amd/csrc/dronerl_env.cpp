// dronerl_env.cpp — library-owned env handles (include/dronerl.h, drl_env_*).
//
// a handle owns the device state of `num_envs` envs on one
// device; the caller owns actions/rewards/dones/obs and passes device pointers;
// every call is asynchronous on the caller's stream (create/destroy allocate
// and free, drl_env_errors synchronises).  The calls forward to the stateless
// entry points (drl_reset / drl_step / drl_obs / drl_decode / drl_encode), so
// the kernels and their validation are shared.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "dronerl_internal.h"

struct drl_env {
    drl_params p;
    drl_layout L;
    int32_t device;
    int64_t num_envs;
    int64_t env_offset;
    uint64_t base_seed;
    int seeded;  // 0: the next reset re-seeds every env (random.seed(base_seed + env_offset + e))
    int32_t since_refill;  // steps since the candidate rings were last topped up (drl_refill)
    drl_state s;
    int32_t* err;
};

// error text shared with dronerl_api.cpp
extern "C" __attribute__((visibility("hidden"))) int drl_internal_fail(const char* msg);

namespace {

// Runs `f` with env->device current, restoring the caller's device after.
template <class F>
int on_device(const drl_env* env, F f) {
    if (!env) return drl_internal_fail("env is NULL");
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return drl_internal_fail("hipGetDevice failed");
    if (prev != env->device && hipSetDevice(env->device) != hipSuccess) return drl_internal_fail("hipSetDevice failed");
    const int rc = f();
    if (prev != env->device) (void)hipSetDevice(prev);
    return rc;
}

int hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return drl_internal_fail(buf);
}

void free_env(drl_env* env) {
    if (!env) return;
    (void)hipFree(env->s.ground);
    (void)hipFree(env->s.drones);
    (void)hipFree(env->s.mt);
    (void)hipFree(env->s.mt_index);
    (void)hipFree(env->err);
    delete env;
}

}  // namespace

extern "C" {

int drl_env_create(const drl_params* p, int32_t device, int64_t num_envs, int64_t env_offset, uint64_t base_seed,
                   drl_env** out) {
    if (!out) return drl_internal_fail("out is NULL");
    *out = nullptr;
    drl_layout L;
    if (drl_layout_query(p, &L)) return -1;
    if (num_envs < 1) return drl_internal_fail("num_envs must be >= 1");
    if (env_offset < 0) return drl_internal_fail("env_offset must be >= 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return drl_internal_fail("device out of range (or no HIP device)");
    drl_env* env = new drl_env();
    env->p = *p;
    env->L = L;
    env->device = device;
    env->num_envs = num_envs;
    env->env_offset = env_offset;
    env->base_seed = base_seed;
    env->seeded = 0;
    env->s.num_envs = num_envs;
    const int rc = on_device(env, [&]() -> int {
        const size_t E = (size_t)num_envs;
        if (hip_check(hipMalloc(&env->s.ground, E * L.ground_stride), "hipMalloc ground") ||
            hip_check(hipMalloc(&env->s.drones, E * L.drone_stride * sizeof(uint32_t)), "hipMalloc drones") ||
            hip_check(hipMalloc(&env->s.mt, E * L.mt_stride * sizeof(uint32_t)), "hipMalloc mt") ||
            hip_check(hipMalloc(&env->s.mt_index, E * sizeof(uint32_t)), "hipMalloc mt_index") ||
            hip_check(hipMalloc(&env->err, sizeof(int32_t)), "hipMalloc err"))
            return -1;
        // defined contents before the first reset (padding bytes included)
        if (hip_check(hipMemset(env->s.ground, 0, E * L.ground_stride), "hipMemset") ||
            hip_check(hipMemset(env->s.drones, 0, E * L.drone_stride * sizeof(uint32_t)), "hipMemset") ||
            hip_check(hipMemset(env->s.mt, 0, E * L.mt_stride * sizeof(uint32_t)), "hipMemset") ||
            hip_check(hipMemset(env->s.mt_index, 0, E * sizeof(uint32_t)), "hipMemset") ||
            hip_check(hipMemset(env->err, 0, sizeof(int32_t)), "hipMemset"))
            return -1;
        return hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    });
    if (rc) {
        free_env(env);
        return -1;
    }
    *out = env;
    return 0;
}

int drl_env_destroy(drl_env* env) {
    if (!env) return 0;
    return on_device(env, [&]() -> int {
        const int rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        free_env(env);
        return rc;
    });
}

int drl_env_seed(drl_env* env, uint64_t base_seed) {
    if (!env) return drl_internal_fail("env is NULL");
    env->base_seed = base_seed;
    env->seeded = 0;
    return 0;
}

int drl_env_reset(drl_env* env, const uint8_t* d_env_mask, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!env->seeded && d_env_mask)
            return drl_internal_fail("the first reset after create/seed must cover every env (mask must be NULL)");
        const int reseed = env->seeded ? 0 : 1;
        if (drl_reset(&env->p, &env->s, reseed, env->base_seed + (uint64_t)env->env_offset, d_env_mask, stream))
            return -1;  // (drl_reset ends with a refill)
        env->seeded = 1;
        env->since_refill = 0;
        return 0;
    });
}

// DRL_STEP_REFILL every layout.refill_every steps
static uint32_t refill_flag(drl_env* env) {
    if (++env->since_refill < env->L.refill_every) return 0u;
    env->since_refill = 0;
    return DRL_STEP_REFILL;
}

int drl_env_step(drl_env* env, const int32_t* d_actions, float* d_rewards, uint8_t* d_dones, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!env->seeded) return drl_internal_fail("step before the first reset");
        return drl_step_ex(&env->p, &env->s, d_actions, d_rewards, d_dones, nullptr, 0, env->err, refill_flag(env),
                           stream);
    });
}

int drl_env_step_obs(drl_env* env, const int32_t* d_actions, float* d_rewards, uint8_t* d_dones, int32_t k,
                     float* d_obs, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!env->seeded) return drl_internal_fail("step before the first reset");
        if (!d_obs) return drl_internal_fail("obs is NULL");
        // store mode as env.step() picks it (drl_default_obs_stream)
        const uint32_t st = env->L.step_group_lanes >= 16 ? DRL_STEP_OBS_STREAM : 0u;
        return drl_step_ex(&env->p, &env->s, d_actions, d_rewards, d_dones, d_obs, k, env->err, refill_flag(env) | st,
                           stream);
    });
}

int drl_env_obs(drl_env* env, int32_t k, float* d_obs, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!env->seeded) return drl_internal_fail("obs before the first reset");
        return drl_obs(&env->p, &env->s, k, d_obs, stream);
    });
}

int drl_env_grid_obs(drl_env* env, float* d_grid, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!env->seeded) return drl_internal_fail("obs before the first reset");
        return drl_grid_obs(&env->p, &env->s, d_grid, stream);
    });
}

int drl_env_get_state(drl_env* env, const drl_state_view* v, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!v) return drl_internal_fail("view is NULL");
        const size_t E = (size_t)env->num_envs, cells = (size_t)env->L.cells;
        if (v->ground && hip_check(drl::launch_ground_unpack(env->s.ground, env->L.ground_stride, v->ground, (int)cells,
                                                             (int64_t)E, stream),
                                   "ground unpack"))
            return -1;
        if (drl_decode(&env->p, &env->s, v->order, v->y, v->x, v->charge, v->carry, stream)) return -1;
        if (v->mt && drl_mt_get(&env->p, &env->s, v->mt, stream)) return -1;
        return 0;
    });
}

int drl_env_set_state(drl_env* env, const drl_state_view* v, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        if (!v || !v->ground || !v->order || !v->y || !v->x || !v->charge || !v->carry || !v->mt)
            return drl_internal_fail("set_state needs every view field");
        const size_t E = (size_t)env->num_envs, cells = (size_t)env->L.cells;
        if (hip_check(drl::launch_ground_pack(v->ground, (int)cells, env->s.ground, env->L.ground_stride, (int64_t)E,
                                              env->err, stream),
                      "ground pack"))
            return -1;
        if (drl_encode(&env->p, &env->s, v->order, v->y, v->x, v->charge, v->carry, stream)) return -1;
        if (drl_mt_set(&env->p, &env->s, v->mt, env->err, stream)) return -1;  // (then a refill)
        env->seeded = 1;
        env->since_refill = 0;
        return 0;
    });
}

int drl_env_state(const drl_env* env, drl_state* s, drl_params* p, drl_layout* L) {
    if (!env) return drl_internal_fail("env is NULL");
    if (s) *s = env->s;
    if (p) *p = env->p;
    if (L) *L = env->L;
    return 0;
}

int drl_env_errors(drl_env* env, int32_t* flags, int32_t clear, hipStream_t stream) {
    return on_device(env, [&]() -> int {
        int32_t h = 0;
        if (hip_check(hipMemcpyAsync(&h, env->err, sizeof h, hipMemcpyDeviceToHost, stream), "err copy") ||
            hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize"))
            return -1;
        if (clear && h && hip_check(hipMemsetAsync(env->err, 0, sizeof(int32_t), stream), "err clear")) return -1;
        if (flags) *flags = h;
        return 0;
    });
}

}  // extern "C"
