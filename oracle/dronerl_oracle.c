/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  NOT PART OF THE PRODUCT.
 *
 * Plain-C restatement of the nyx-ai/droneRL `torch_impl` environment
 * (the parity target named by BASELINE.json), written from reading the
 * reference as text.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or as the
 * timed CPU baseline).  The product path (dronerl_amd/libdronerl.so) never
 * links, loads or calls it.
 *
 * Parity is pinned two ways (see tests/test_oracle_golden.py):
 *   - the reference's own golden tests, restated as data in tests/golden/
 *     (test_windowedgridview.py matrices, test_env_single_drone.py and
 *     test_env_multiple_drones.py asserted vectors, jax_tests/test_env.py
 *     RNG-free known answers);
 *   - trajectories produced by importing /root/reference/torch_impl in the
 *     build container (oracle/gen_golden.py -> tests/golden/traj_*.npz).
 *
 * What is restated (file:line in /root/reference):
 *   CPython random (stdlib, Modules/_randommodule.c + Lib/random.py 3.10):
 *     init_genrand / init_by_array / genrand_uint32, getrandbits(k<=32),
 *     _randbelow_with_getrandbits (random.py:239-247), shuffle (random.py:380-395),
 *     sample (random.py:480-504, both the pool and the set branch).
 *   torch_impl/env/env.py
 *     spawn_objects            :58-66
 *     reset                    :68-101
 *     step                     :112-215
 *     _pick_packets_after_respawn :217-224
 *     _find_respawn_position   :226-233
 *   torch_impl/env/wrappers.py
 *     BaseGridView._create_base_grid :10-31
 *     WindowedGridView.observation   :55-73
 *
 * The restatement deliberately mirrors the reference's dict-based control flow
 * (ordered drone "dict", crash lists A and B, crashed-location list) rather
 * than the GPU kernel's lane-parallel formulation, so the two are independent.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* CPython MT19937                                                            */
/* ------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t mt[MT_N];
    int32_t index; /* CPython's `index`; 624 => next draw twists */
} orc_mt;

static void mt_init_genrand(orc_mt* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->index = MT_N;
}

static void mt_init_by_array(orc_mt* s, const uint32_t* key, int keylen) {
    mt_init_genrand(s, 19650218u);
    int i = 1, j = 0;
    int k = (MT_N > keylen) ? MT_N : keylen;
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
        if (j >= keylen) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
    s->index = MT_N;
}

/* random.seed(int) for a non-negative integer < 2**64: key = 32-bit words of
 * |a|, little-endian; a == 0 gives key [0]. */
void orc_mt_seed(orc_mt* s, uint64_t seed) {
    uint32_t key[2];
    int keylen;
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
    keylen = key[1] ? 2 : 1;
    mt_init_by_array(s, key, keylen);
}

static void mt_twist(orc_mt* s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    uint32_t* mt = s->mt;
    int kk;
    uint32_t y;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    s->index = 0;
}

uint32_t orc_mt_genrand(orc_mt* s) {
    if (s->index >= MT_N) mt_twist(s);
    uint32_t y = s->mt[s->index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static int bit_length(uint32_t n) {
    int k = 0;
    while (n) { k++; n >>= 1; }
    return k;
}

/* getrandbits(k), 1 <= k <= 32 */
uint32_t orc_getrandbits(orc_mt* s, int k) { return orc_mt_genrand(s) >> (32 - k); }

/* Random._randbelow_with_getrandbits (random.py:239-247) */
uint32_t orc_randbelow(orc_mt* s, uint32_t n) {
    if (!n) return 0;
    int k = bit_length(n);
    uint32_t r = orc_getrandbits(s, k);
    while (r >= n) r = orc_getrandbits(s, k);
    return r;
}

/* Random.shuffle (random.py:380-395), on an int32 list */
void orc_shuffle(orc_mt* s, int32_t* x, int32_t n) {
    for (int32_t i = n - 1; i >= 1; i--) {
        uint32_t j = orc_randbelow(s, (uint32_t)(i + 1));
        int32_t t = x[i];
        x[i] = x[j];
        x[j] = t;
    }
}

/* Random.sample(population, k) (random.py:480-504); returns 0 or -1 on bad k. */
int orc_sample(orc_mt* s, const int32_t* pop, int32_t n, int32_t k, int32_t* result) {
    if (k < 0 || k > n) return -1;
    int32_t setsize = 21;
    if (k > 5) setsize += (int32_t)pow(4.0, ceil(log((double)(k * 3)) / log(4.0)));
    if (n <= setsize) {
        int32_t* pool = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
        memcpy(pool, pop, sizeof(int32_t) * (size_t)n);
        for (int32_t i = 0; i < k; i++) {
            uint32_t j = orc_randbelow(s, (uint32_t)(n - i));
            result[i] = pool[j];
            pool[j] = pool[n - i - 1];
        }
        free(pool);
    } else {
        int32_t* selected = (int32_t*)malloc(sizeof(int32_t) * (size_t)(k > 0 ? k : 1));
        int32_t nsel = 0;
        for (int32_t i = 0; i < k; i++) {
            uint32_t j;
            for (;;) {
                j = orc_randbelow(s, (uint32_t)n);
                int seen = 0;
                for (int32_t q = 0; q < nsel; q++)
                    if (selected[q] == (int32_t)j) { seen = 1; break; }
                if (!seen) break;
            }
            selected[nsel++] = (int32_t)j;
            result[i] = pop[j];
        }
        free(selected);
    }
    return 0;
}

/* CPython getstate()/setstate() interchange: 624 words + index */
void orc_mt_get(const orc_mt* s, uint32_t* words625) {
    memcpy(words625, s->mt, sizeof(uint32_t) * MT_N);
    words625[MT_N] = (uint32_t)s->index;
}
void orc_mt_set(orc_mt* s, const uint32_t* words625) {
    memcpy(s->mt, words625, sizeof(uint32_t) * MT_N);
    s->index = (int32_t)words625[MT_N];
}
size_t orc_mt_sizeof(void) { return sizeof(orc_mt); }

/* ------------------------------------------------------------------------- */
/* torch_impl DeliveryDrones                                                  */
/* ------------------------------------------------------------------------- */
enum { OBJ_EMPTY = 0, OBJ_SKYSCRAPER = 2, OBJ_STATION = 3, OBJ_DROPZONE = 4, OBJ_PACKET = 5 };

/* env.py:26 ACTION_TO_DIRECTION, (dy, dx) */
static const int DIR_Y[5] = {0, 1, 0, -1, 0};
static const int DIR_X[5] = {-1, 0, 1, 0, 0};

typedef struct {
    int32_t side;      /* G */
    int32_t n_drones;  /* N */
    int32_t charge;
    int32_t discharge;
    int32_t packets_factor, dropzones_factor, stations_factor, skyscrapers_factor;
    double pickup_reward, delivery_reward, crash_reward, charge_reward;
} orc_params;

typedef struct {
    orc_params p;
    int32_t n_order;   /* number of drones in the dict (== N between calls) */
    uint8_t* ground;   /* [G*G] object code per cell (the 4 object dicts are disjoint) */
    int32_t* order;    /* [N] drone index at dict position (insertion order O) */
    int32_t* pos;      /* [N] cell (y*G+x) of drone index */
    int32_t* charge;   /* [N] */
    uint8_t* packet;   /* [N] */
    int32_t* scratch;  /* work lists */
    orc_mt rng;
} orc_env;

size_t orc_env_sizeof(void) { return sizeof(orc_env); }

orc_env* orc_env_create(const orc_params* p) {
    if (p->side <= 0 || p->n_drones <= 0) return NULL;
    orc_env* e = (orc_env*)calloc(1, sizeof(orc_env));
    e->p = *p;
    int GG = p->side * p->side, N = p->n_drones;
    e->ground = (uint8_t*)calloc((size_t)GG, 1);
    e->order = (int32_t*)calloc((size_t)N, sizeof(int32_t));
    e->pos = (int32_t*)calloc((size_t)N, sizeof(int32_t));
    e->charge = (int32_t*)calloc((size_t)N, sizeof(int32_t));
    e->packet = (uint8_t*)calloc((size_t)N, 1);
    e->scratch = (int32_t*)calloc((size_t)(4 * GG + 8 * N + 16), sizeof(int32_t));
    orc_mt_seed(&e->rng, 0);
    return e;
}

void orc_env_destroy(orc_env* e) {
    if (!e) return;
    free(e->ground); free(e->order); free(e->pos); free(e->charge); free(e->packet); free(e->scratch);
    free(e);
}

orc_mt* orc_env_rng(orc_env* e) { return &e->rng; }

/* env.py:217-224 */
static void pick_packets_after_respawn(orc_env* e) {
    for (int32_t q = 0; q < e->n_order; q++) {
        int32_t d = e->order[q];
        int32_t c = e->pos[d];
        if (!e->packet[d] && e->ground[c] == OBJ_PACKET) {
            e->packet[d] = 1;
            e->ground[c] = OBJ_EMPTY;
        }
    }
}

/* env.py:58-66 spawn_objects: shuffle, then pop num_obj from the end */
static int spawn_objects(orc_env* e, int32_t* avail, int32_t* n_avail, int32_t num, uint8_t code) {
    if (*n_avail < num) return -1;
    orc_shuffle(&e->rng, avail, *n_avail);
    for (int32_t i = 0; i < num; i++) {
        int32_t cell = avail[--(*n_avail)];
        e->ground[cell] = code;
    }
    return 0;
}

/* env.py:68-101.  Returns 0, or -1 when the grid cannot hold the objects
 * (the reference raises ValueError from spawn_objects / sample). */
int orc_reset(orc_env* e) {
    const int32_t G = e->p.side, N = e->p.n_drones, GG = G * G;
    int32_t* avail = e->scratch;
    int32_t* sample = e->scratch + GG;
    memset(e->ground, 0, (size_t)GG);
    /* [(x, y) for x in range(G) for y in range(G)] -> element i is key (i//G, i%G),
     * read everywhere else as (row, col): cell id i. */
    for (int32_t i = 0; i < GG; i++) avail[i] = i;
    int32_t n = GG;
    if (spawn_objects(e, avail, &n, e->p.skyscrapers_factor * N, OBJ_SKYSCRAPER)) return -1;
    if (orc_sample(&e->rng, avail, n, N, sample)) return -1;
    for (int32_t i = 0; i < N; i++) {
        e->order[i] = i;
        e->pos[i] = sample[i];
        e->charge[i] = 100;
        e->packet[i] = 0;
    }
    e->n_order = N;
    if (spawn_objects(e, avail, &n, e->p.packets_factor * N, OBJ_PACKET)) return -1;
    if (spawn_objects(e, avail, &n, e->p.dropzones_factor * N, OBJ_DROPZONE)) return -1;
    if (spawn_objects(e, avail, &n, e->p.stations_factor * N, OBJ_STATION)) return -1;
    pick_packets_after_respawn(e);
    return 0;
}

/* env.py:226-233.  mask: 1 = blocked; n_blocked: how many cells are.
 * Returns the cell, or -1 when every cell is blocked: the reference's loop
 * would spin forever there (the kernel raises DRL_ERR_NO_FREE_CELL). */
static int32_t find_respawn_position(orc_env* e, const uint8_t* mask, int32_t n_blocked) {
    const uint32_t G = (uint32_t)e->p.side;
    if (n_blocked >= (int32_t)(G * G)) return -1;
    for (;;) {
        uint32_t y = orc_randbelow(&e->rng, G); /* randint(0, G-1) */
        uint32_t x = orc_randbelow(&e->rng, G);
        int32_t c = (int32_t)(y * G + x);
        if (!mask[c]) return c;
    }
}

/* env.py:112-215.  actions[N] by drone index; rewards[N]/dones[N] by drone
 * index.  Returns 0, -1 on an action index Python would reject, or -2 when a
 * respawn finds every cell blocked (the reference loops forever there). */
int orc_step(orc_env* e, const int32_t* actions, double* rewards, uint8_t* dones) {
    const int32_t G = e->p.side, N = e->p.n_drones, GG = G * G;
    int32_t* new_at = e->scratch;               /* [GG] drone+1 claiming a cell (new_drones) */
    int32_t* new_keys = e->scratch + GG;        /* [N] insertion order of new_drones (cells) */
    int32_t* crashed = new_keys + N;            /* [2N] crashed_drones */
    int32_t* crashed_locs = crashed + 2 * N;    /* [3N] crashed_drone_locations */
    uint8_t* mask = (uint8_t*)(crashed_locs + 3 * N); /* [GG] */
    int32_t n_new = 0, n_crashed = 0, n_locs = 0;
    int32_t nb_drop = 0, nb_pack = 0;

    for (int32_t d = 0; d < N; d++) { rewards[d] = 0.0; dones[d] = 0; }
    for (int32_t d = 0; d < N; d++) {
        int32_t a = actions[d];
        if (a < -5 || a > 4) return -1;        /* IndexError in the reference */
    }
    memset(new_at, 0, sizeof(int32_t) * (size_t)GG);

    /* move all drones (env.py:124-140), in dict order */
    for (int32_t q = 0; q < e->n_order; q++) {
        int32_t d = e->order[q];
        int32_t a = actions[d];
        if (a < 0) a += 5;                     /* Python negative list index */
        int32_t y = e->pos[d] / G, x = e->pos[d] % G;
        int32_t ny = y + DIR_Y[a], nx = x + DIR_X[a];
        if (0 <= ny && ny < G && 0 <= nx && nx < G) {
            int32_t c = ny * G + nx;
            if (new_at[c]) {
                crashed[n_crashed++] = d;
                crashed_locs[n_locs++] = c;
            } else {
                new_at[c] = d + 1;
                new_keys[n_new++] = c;
            }
        } else {
            crashed[n_crashed++] = d;
        }
    }

    /* drones that did not crash yet (env.py:143-172), new_drones order */
    for (int32_t q = 0; q < n_new; q++) {
        int32_t c = new_keys[q];
        int32_t d = new_at[c] - 1;
        int in_crashed = 0;
        for (int32_t t = 0; t < n_crashed; t++)
            if (crashed[t] == d) { in_crashed = 1; break; }
        if (in_crashed) continue;
        uint8_t obj = e->ground[c];
        if (obj == OBJ_STATION) {
            int32_t v = e->charge[d] + e->p.charge;
            e->charge[d] = v < 100 ? v : 100;
            rewards[d] = e->p.charge_reward;
        } else {
            e->charge[d] -= e->p.discharge;
            if (e->charge[d] <= 0) crashed_locs[n_locs++] = c;
        }
        if (obj == OBJ_PACKET && !e->packet[d]) {
            rewards[d] = e->p.pickup_reward;
            e->packet[d] = 1;
            e->ground[c] = OBJ_EMPTY;
        } else if (obj == OBJ_DROPZONE && e->packet[d]) {
            rewards[d] = e->p.delivery_reward;
            e->packet[d] = 0;
            e->ground[c] = OBJ_EMPTY;
            nb_drop++;
            nb_pack++;
        }
        if (obj == OBJ_SKYSCRAPER) crashed_locs[n_locs++] = c;
    }

    /* crash-location sweep (env.py:177-181) */
    for (int32_t t = 0; t < n_locs; t++) {
        int32_t c = crashed_locs[t];
        if (new_at[c]) {
            crashed[n_crashed++] = new_at[c] - 1;
            new_at[c] = 0;  /* del new_drones[c]; dict order of the rest is kept */
        }
    }

    /* self.drones = new_drones (env.py:183) */
    int32_t no = 0;
    for (int32_t q = 0; q < n_new; q++) {
        int32_t c = new_keys[q];
        if (new_at[c]) {
            int32_t d = new_at[c] - 1;
            e->order[no++] = d;
            e->pos[d] = c;
        }
    }
    e->n_order = no;

    /* respawn crashed drones (env.py:186-195); mask = drones | skyscrapers */
    int32_t n_blocked = 0;
    for (int32_t c = 0; c < GG; c++) n_blocked += mask[c] = (e->ground[c] == OBJ_SKYSCRAPER);
    for (int32_t q = 0; q < e->n_order; q++) {
        int32_t c = e->pos[e->order[q]];
        n_blocked += !mask[c];
        mask[c] = 1;
    }
    int no_free = 0;
    for (int32_t t = 0; t < n_crashed; t++) {
        int32_t d = crashed[t];
        e->charge[d] = 100;
        if (e->packet[d]) {
            nb_pack++;
            e->packet[d] = 0;
        }
        rewards[d] = e->p.crash_reward;
        dones[d] = 1;
        int32_t c = find_respawn_position(e, mask, n_blocked);
        if (c < 0) { no_free = 1; break; }
        e->pos[d] = c;
        e->order[e->n_order++] = d;
        mask[c] = 1;
        n_blocked++;
    }

    /* respawn used packets and dropzones (env.py:198-210) */
    n_blocked = 0;
    for (int32_t c = 0; c < GG; c++) n_blocked += mask[c] = (e->ground[c] != OBJ_EMPTY);
    for (int32_t t = 0; t < nb_pack && !no_free; t++) {
        int32_t c = find_respawn_position(e, mask, n_blocked);
        if (c < 0) { no_free = 1; break; }
        e->ground[c] = OBJ_PACKET;
        mask[c] = 1;
        n_blocked++;
    }
    for (int32_t t = 0; t < nb_drop && !no_free; t++) {
        int32_t c = find_respawn_position(e, mask, n_blocked);
        if (c < 0) { no_free = 1; break; }
        e->ground[c] = OBJ_DROPZONE;
        mask[c] = 1;
        n_blocked++;
    }
    if (no_free) return -2; /* the reference never returns from this step */

    pick_packets_after_respawn(e);
    return 0;
}

/* WindowedGridView.observation (wrappers.py:10-31, 55-73) for drone indices
 * 0..k-1 into out[k][2r+1][2r+1][6] (float32, as the DQN consumes it:
 * torch_impl/agents/dqn.py:81).  charge channel = (float)(charge / 100) in
 * double, exactly as the f32 grid stores the Python float. */
void orc_obs(const orc_env* e, int32_t radius, int32_t k, float* out) {
    const int32_t G = e->p.side, W = 2 * radius + 1;
    for (int32_t d = 0; d < k; d++) {
        int32_t py = e->pos[d] / G, px = e->pos[d] % G;
        float* o = out + (size_t)d * W * W * 6;
        for (int32_t wy = 0; wy < W; wy++) {
            for (int32_t wx = 0; wx < W; wx++) {
                float* v = o + (wy * W + wx) * 6;
                int32_t y = py + wy - radius, x = px + wx - radius;
                for (int ch = 0; ch < 6; ch++) v[ch] = 0.0f;
                if (y < 0 || y >= G || x < 0 || x >= G) {
                    v[5] = 1.0f;
                    continue;
                }
                int32_t c = y * G + x;
                uint8_t obj = e->ground[c];
                if (obj == OBJ_PACKET) v[1] = 1.0f;
                if (obj == OBJ_DROPZONE) v[2] = 1.0f;
                if (obj == OBJ_STATION) v[3] = 1.0f;
                if (obj == OBJ_SKYSCRAPER) v[5] = 1.0f;
                for (int32_t q = 0; q < e->n_order; q++) {
                    int32_t dd = e->order[q];
                    if (e->pos[dd] == c) {
                        v[0] = 1.0f;
                        if (e->packet[dd]) v[1] = 1.0f;
                        v[4] = (float)((double)e->charge[dd] / 100.0);
                    }
                }
            }
        }
    }
}

/* State interchange.  order[N]: drone index per dict position; y/x/charge/
 * packet by drone index; ground[G*G]; mt625 = CPython getstate() words. */
void orc_get_state(const orc_env* e, uint8_t* ground, int32_t* order, int32_t* y, int32_t* x,
                   int32_t* charge, uint8_t* packet, uint32_t* mt625) {
    const int32_t G = e->p.side, N = e->p.n_drones;
    if (ground) memcpy(ground, e->ground, (size_t)(G * G));
    for (int32_t d = 0; d < N; d++) {
        if (order) order[d] = e->order[d];
        if (y) y[d] = e->pos[d] / G;
        if (x) x[d] = e->pos[d] % G;
        if (charge) charge[d] = e->charge[d];
        if (packet) packet[d] = e->packet[d];
    }
    if (mt625) orc_mt_get(&e->rng, mt625);
}

void orc_set_state(orc_env* e, const uint8_t* ground, const int32_t* order, const int32_t* y,
                   const int32_t* x, const int32_t* charge, const uint8_t* packet,
                   const uint32_t* mt625) {
    const int32_t G = e->p.side, N = e->p.n_drones;
    if (ground) memcpy(e->ground, ground, (size_t)(G * G));
    for (int32_t d = 0; d < N; d++) {
        if (order) e->order[d] = order[d];
        if (y && x) e->pos[d] = y[d] * G + x[d];
        if (charge) e->charge[d] = charge[d];
        if (packet) e->packet[d] = packet[d];
    }
    e->n_order = N;
    if (mt625) orc_mt_set(&e->rng, mt625);
}

/* ------------------------------------------------------------------------- */
/* Synthetic random actions shared with the GPU bench (counter-based, so any  */
/* env subset regenerates the identical stream).                              */
/* ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int32_t orc_synth_action(uint64_t seed, uint64_t step, uint64_t env, uint32_t n_drones, uint32_t drone) {
    uint64_t ctr = (step << 40) ^ (env << 8) ^ (uint64_t)drone;
    (void)n_drones;
    uint64_t h = splitmix64(seed ^ splitmix64(ctr));
    return (int32_t)(((h >> 32) * 5ull) >> 32);
}

/* ------------------------------------------------------------------------- */
/* Batched rollout (CPU baseline + bulk parity): E independent envs with      */
/* env e seeded random.seed(seed0 + env_offset + e), `steps` synthetic-action */
/* steps each.  Optional outputs per env: final ground / drone vectors and    */
/* reward/done sums.  nthreads >= 1 static env partition.                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    const orc_params* p;
    int64_t e0, e1, env_offset, steps;
    uint64_t seed0, action_seed;
    uint8_t* ground;   /* [E][G*G] or NULL */
    int32_t* order;    /* [E][N] or NULL */
    int32_t* y; int32_t* x; int32_t* charge; uint8_t* packet;
    uint32_t* mt625;   /* [E][625] or NULL */
    double* reward_sum; /* [E] or NULL */
    int64_t* done_sum;  /* [E] or NULL */
    int32_t obs_k, radius; /* >0: also compute the WindowedGridView obs of drones 0..obs_k-1 every step */
    double obs_checksum;
    int status;
} rollout_job;

static void* rollout_worker(void* arg) {
    rollout_job* j = (rollout_job*)arg;
    const int32_t N = j->p->n_drones, GG = j->p->side * j->p->side;
    orc_env* e = orc_env_create(j->p);
    int32_t* act = (int32_t*)malloc(sizeof(int32_t) * (size_t)N);
    double* rew = (double*)malloc(sizeof(double) * (size_t)N);
    uint8_t* dn = (uint8_t*)malloc((size_t)N);
    const int32_t W = 2 * j->radius + 1;
    float* ob = j->obs_k > 0 ? (float*)malloc(sizeof(float) * (size_t)j->obs_k * W * W * 6) : NULL;
    j->status = 0;
    j->obs_checksum = 0.0;
    for (int64_t i = j->e0; i < j->e1; i++) {
        uint64_t genv = (uint64_t)(j->env_offset + i);
        orc_mt_seed(&e->rng, j->seed0 + genv);
        if (orc_reset(e)) { j->status = -1; break; }
        double rs = 0.0;
        int64_t ds = 0;
        for (int64_t s = 0; s < j->steps; s++) {
            for (int32_t d = 0; d < N; d++) act[d] = orc_synth_action(j->action_seed, (uint64_t)s, genv, (uint32_t)N, (uint32_t)d);
            orc_step(e, act, rew, dn);
            for (int32_t d = 0; d < N; d++) { rs += rew[d]; ds += dn[d]; }
            if (ob) {
                orc_obs(e, j->radius, j->obs_k, ob);
                j->obs_checksum += ob[(s * 7) % (j->obs_k * W * W * 6)];
            }
        }
        orc_get_state(e, j->ground ? j->ground + i * GG : NULL, j->order ? j->order + i * N : NULL,
                      j->y ? j->y + i * N : NULL, j->x ? j->x + i * N : NULL,
                      j->charge ? j->charge + i * N : NULL, j->packet ? j->packet + i * N : NULL,
                      j->mt625 ? j->mt625 + i * 625 : NULL);
        if (j->reward_sum) j->reward_sum[i] = rs;
        if (j->done_sum) j->done_sum[i] = ds;
    }
    free(act); free(rew); free(dn); free(ob);
    orc_env_destroy(e);
    return NULL;
}

int orc_rollout(const orc_params* p, int64_t E, int64_t env_offset, uint64_t seed0, uint64_t action_seed,
                int64_t steps, int32_t nthreads, int32_t obs_k, int32_t radius, uint8_t* ground, int32_t* order,
                int32_t* y, int32_t* x, int32_t* charge, uint8_t* packet, uint32_t* mt625, double* reward_sum,
                int64_t* done_sum) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    rollout_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        rollout_job* j = &jobs[t];
        j->p = p;
        j->e0 = E * t / nthreads;
        j->e1 = E * (t + 1) / nthreads;
        j->env_offset = env_offset;
        j->steps = steps;
        j->seed0 = seed0;
        j->action_seed = action_seed;
        j->ground = ground; j->order = order; j->y = y; j->x = x; j->charge = charge; j->packet = packet;
        j->mt625 = mt625; j->reward_sum = reward_sum; j->done_sum = done_sum;
        j->obs_k = obs_k; j->radius = radius;
        if (nthreads == 1) rollout_worker(j);
        else pthread_create(&th[t], NULL, rollout_worker, j);
    }
    int st = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].status) st = jobs[t].status;
    }
    return st;
}

/* ------------------------------------------------------------------------- */
/* Multi-env container for per-step parity checks at thousands of envs.      */
/* ------------------------------------------------------------------------- */
typedef struct {
    orc_params p;
    int64_t E;
    orc_env** envs;
} orc_multi;

orc_multi* orc_multi_create(const orc_params* p, int64_t E) {
    orc_multi* m = (orc_multi*)calloc(1, sizeof(orc_multi));
    m->p = *p;
    m->E = E;
    m->envs = (orc_env**)calloc((size_t)E, sizeof(orc_env*));
    for (int64_t i = 0; i < E; i++) m->envs[i] = orc_env_create(p);
    return m;
}

void orc_multi_destroy(orc_multi* m) {
    if (!m) return;
    for (int64_t i = 0; i < m->E; i++) orc_env_destroy(m->envs[i]);
    free(m->envs);
    free(m);
}

/* seeds[E] (NULL: continue streams); returns -1 if any reset fails */
int orc_multi_reset(orc_multi* m, const uint64_t* seeds) {
    int st = 0;
    for (int64_t i = 0; i < m->E; i++) {
        if (seeds) orc_mt_seed(&m->envs[i]->rng, seeds[i]);
        if (orc_reset(m->envs[i])) st = -1;
    }
    return st;
}

typedef struct {
    orc_multi* m;
    int64_t e0, e1;
    const int32_t* actions;
    double* rewards;
    uint8_t* dones;
    int status;
} multi_job;

static void* multi_step_worker(void* arg) {
    multi_job* j = (multi_job*)arg;
    const int32_t N = j->m->p.n_drones;
    j->status = 0;
    for (int64_t i = j->e0; i < j->e1; i++)
        {
            int r = orc_step(j->m->envs[i], j->actions + i * N, j->rewards + i * N, j->dones + i * N);
            if (r && (!j->status || r == -2)) j->status = r;
        }
    return NULL;
}

int orc_multi_step(orc_multi* m, const int32_t* actions, double* rewards, uint8_t* dones, int32_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    multi_job jobs[64];
    for (int t = 0; t < nthreads; t++) {
        jobs[t].m = m;
        jobs[t].e0 = m->E * t / nthreads;
        jobs[t].e1 = m->E * (t + 1) / nthreads;
        jobs[t].actions = actions;
        jobs[t].rewards = rewards;
        jobs[t].dones = dones;
        if (nthreads == 1) multi_step_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, multi_step_worker, &jobs[t]);
    }
    int st = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].status && (!st || jobs[t].status == -2)) st = jobs[t].status;
    }
    return st;
}

void orc_multi_get_state(const orc_multi* m, uint8_t* ground, int32_t* order, int32_t* y, int32_t* x,
                         int32_t* charge, uint8_t* packet, uint32_t* mt625) {
    const int32_t N = m->p.n_drones, GG = m->p.side * m->p.side;
    for (int64_t i = 0; i < m->E; i++)
        orc_get_state(m->envs[i], ground ? ground + i * GG : NULL, order ? order + i * N : NULL,
                      y ? y + i * N : NULL, x ? x + i * N : NULL, charge ? charge + i * N : NULL,
                      packet ? packet + i * N : NULL, mt625 ? mt625 + i * 625 : NULL);
}

void orc_multi_set_state(orc_multi* m, const uint8_t* ground, const int32_t* order, const int32_t* y,
                         const int32_t* x, const int32_t* charge, const uint8_t* packet, const uint32_t* mt625) {
    const int32_t N = m->p.n_drones, GG = m->p.side * m->p.side;
    for (int64_t i = 0; i < m->E; i++)
        orc_set_state(m->envs[i], ground ? ground + i * GG : NULL, order ? order + i * N : NULL,
                      y ? y + i * N : NULL, x ? x + i * N : NULL, charge ? charge + i * N : NULL,
                      packet ? packet + i * N : NULL, mt625 ? mt625 + i * 625 : NULL);
}

/* obs of drone indices 0..k-1 for every env: out[E][k][W][W][6] */
void orc_multi_obs(const orc_multi* m, int32_t radius, int32_t k, float* out) {
    const int32_t W = 2 * radius + 1;
    for (int64_t i = 0; i < m->E; i++) orc_obs(m->envs[i], radius, k, out + i * (int64_t)k * W * W * 6);
}
