/*
 * spgg_abi.h — C ABI of libspgg_hip.so, the MI355X (gfx950) implementation of
 * the SPGG per-iteration hot path.
 *
 * Replaces, per executed iteration of the reference's run loop:
 *   - payoff of the 5 overlapping groups      src/model/spgg.py:23-36, 230-279, 373-378
 *   - state representation (reputation/action) src/model/spgg.py:281-317, 409, 423
 *   - eps-greedy action select                 src/model/algorithms.py:102-110 (+ copies)
 *   - reputation update                        src/model/spgg.py:319-323, 413-416
 *   - reward                                   src/model/spgg.py:424-427
 *   - TD update of the RL operator             src/model/algorithms.py:112-341
 *       Q-learning :112-133, SARSA :152-178 (+ spgg.py:432-438), Expected SARSA
 *       :191-234, Double Q-learning :285-341 (+ spgg.py:496-505)
 *   - diagnostic TD + neighbor-influence term  src/model/spgg.py:445-509
 *   - per-step history reductions              src/model/spgg.py:380-394, 418-420, 511-545, 561-592
 * The reference has no native layer; this ABI is what its Python would bind
 * (see INTEGRATION.md for the ctypes binding used by the drop-in SPGG class).
 *
 * Conventions: every function returns 0 on success, a negative SPGG_E* code on
 * failure (detail in spgg_last_error).  No C++ exception crosses the ABI.
 * One iteration is ONE kernel launch over all replicas (plus one prologue launch
 * before iteration 1).  In MT19937 mode a generator kernel produces the draw
 * records of 8 iterations per launch (SPGG_MT_CHUNK) on a second stream, one
 * chunk ahead of the steps (ordered by events; spgg_set_draw_stream).
 * Buffers are DEVICE pointers owned by the caller (e.g. torch tensors); the
 * library only allocates its per-replica parameter table and frees it in
 * spgg_destroy.  A context is bound to one device and is not thread-safe.
 * spgg_step / spgg_flush only ENQUEUE work on the given HIP stream.
 */
#ifndef SPGG_ABI_H
#define SPGG_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPGG_ABI_VERSION 11

#define SPGG_OK 0
#define SPGG_E_ARG (-1)     /* bad argument / shape */
#define SPGG_E_STATE (-2)   /* call order (e.g. step before bind) */
#define SPGG_E_HIP (-3)     /* HIP runtime error */

/* state representation (spgg.py:289-310) */
#define SPGG_STATE_REPUTATION 0
#define SPGG_STATE_ACTION 1

/* RL operator (algorithms.py:344-383) */
#define SPGG_ALG_QLEARNING 0
#define SPGG_ALG_SARSA 1
#define SPGG_ALG_EXPECTED_SARSA 2
#define SPGG_ALG_DOUBLE_Q 3

/* random stream used by the eps-greedy selects */
#define SPGG_RNG_INJECT 0   /* caller fills the draw planes per step (host MT19937 etc.) */
#define SPGG_RNG_MT19937 1  /* device MT19937, bit-identical to numpy.random.RandomState */
#define SPGG_RNG_PHILOX 2   /* counter-based Philox2x32-10 keyed by (seed, replica), counter (agent pair, step) */

/* Per-step history record: stats[rep][stripe][t][SPGG_NSTAT] (float64), t = 0 ..
 * iterations+1, stripe = 0 .. spgg_stat_stripes()-1.  A slot's value is the SUM of its
 * stripes, except SPGG_ST_GMAX: the MAX.  Integer counts are stored exactly as float64.
 * The slots marked (derived) are filled by spgg_history_finalize from the counted ones
 * (slot 0 holds the group composition of S_1, written by iteration 1's prologue). */
enum {
  SPGG_ST_NCOOP = 0,      /* #S_t==0 at iteration start (spgg.py:383)            */
  SPGG_ST_SUMP = 1,       /* sum P (derived)             (spgg.py:388)            */
  SPGG_ST_SUMP_C = 2,     /* sum P over S_t==0 (derived) (spgg.py:389)            */
  SPGG_ST_SUMP_D = 3,     /* sum P over S_t==1 (derived) (spgg.py:390)            */
  SPGG_ST_SUMR = 4,       /* sum R_t                     (spgg.py:394)            */
  SPGG_ST_SW_CD = 5,      /* switches C->D               (spgg.py:419)            */
  SPGG_ST_SW_DC = 6,      /* switches D->C (derived)     (spgg.py:420)            */
  SPGG_ST_SUM_WPP = 7,    /* sum w_P*P (derived)         (spgg.py:425)            */
  SPGG_ST_SUM_WRR = 8,    /* sum w_rep*rep_reward (derived) (spgg.py:426)         */
  SPGG_ST_SUM_REW_C = 9,  /* sum reward over a==0        (spgg.py:542)            */
  SPGG_ST_SUM_REW_D = 10, /* sum reward over a==1 (derived) (spgg.py:543)         */
  SPGG_ST_SUM_RATIO_C = 11, /* sum rep-reward ratio over a==0 (spgg.py:533-535)   */
  SPGG_ST_GC0 = 12,       /* 12..17: #agents with d defectors in 5-pt group (spgg.py:586-592) */
  SPGG_ST_NMD_POS = 18,   /* #agents with max_diff > 0   (spgg.py:521)            */
  SPGG_ST_NMD_POS2 = 19,  /* ... whose best neighbor is second order (spgg.py:520-523) */
  SPGG_ST_SUM_PCT = 20,   /* sum NI percent              (spgg.py:512-513)        */
  SPGG_ST_SUMQ = 21,      /* 21..24: sum Q[:,:,s,a] after NI, index 2s+a (spgg.py:562-565) */
  SPGG_ST_SUMQ_C = 25,    /* 25..28: ... over prev_S==0  (spgg.py:568-577)        */
  SPGG_ST_SUMQ_D = 29,    /* 29..32: ... over prev_S==1  (spgg.py:579-583)        */
  SPGG_ST_GMAX = 33,      /* global max |diff| (float64 bits, atomic max) (spgg.py:488) */
  SPGG_NSTAT = 34
};

typedef struct spgg_ctx spgg_ctx;

typedef struct {
  int32_t device;        /* HIP device ordinal */
  int32_t n_rep;         /* replicas in the batch (independent lattices) */
  int32_t L;             /* lattice side */
  int32_t second_order;  /* use_second_order (M=2) */
  int32_t state_mode;    /* SPGG_STATE_* */
  int32_t rng_mode;      /* SPGG_RNG_* */
  int32_t iterations;    /* capacity: stats/eps tables hold iterations+2 slots */
  int32_t rep_int8;      /* 1: R buffers hold int8 multiples of each replica's rep_unit
                            (exact when gains/bounds are dyadic multiples, see below) */
  int32_t algorithm;     /* SPGG_ALG_* */
  int32_t batch_reps;    /* replicas of the whole batch whose buffers this context's
                            replicas are a slice of (>= n_rep; 0 = n_rep).  The tiling
                            (agents per thread, tile shape, border-record layout, history
                            stripes) is chosen from it, so every context of one batch
                            (replica groups on separate streams) gets the same layout. */
} spgg_config;

/* Per-replica constants, precomputed by the host in the reference's own
 * (Python float) arithmetic so the device reproduces it bit for bit. */
typedef struct {
  double rc;          /* r*c                       (spgg.py:256)  */
  double cost;        /*                           (spgg.py:256)  */
  double norm_min;    /* r-5                       (spgg.py:149)  */
  double norm_den;    /* 4r-(r-5)                  (spgg.py:377)  */
  double w_p;         /* reward_weight_payoff      (spgg.py:427)  */
  double w_rep;       /* 1-w_P                     (spgg.py:108)  */
  double alpha;       /* TD learning rate (algorithm's)  (algorithms.py:131) */
  double gamma;       /* TD discount (algorithm's)       (algorithms.py:128) */
  double diag_alpha;  /* SPGG.alpha for the NI percent   (spgg.py:475,512)  */
  double diag_gamma;  /* SPGG.gamma for the diag TD      (spgg.py:473)      */
  double kappa;       /* influence_factor          (spgg.py:489)  */
  double lambda_eps;  /* lambda_epsilon            (spgg.py:489)  */
  double rep_gain_c;  /* reputation gain on C      (spgg.py:321)  */
  double neg_delta_r_d; /* -delta_R_D              (spgg.py:321)  */
  double r_min;
  double r_max;
  uint64_t seed;      /* Philox key (SPGG_RNG_PHILOX only) */
  uint64_t stream_id; /* Philox stream: the caller's GLOBAL replica index (BatchEngine: its
                         replica_offset, a rank's shard start, + k), so a replica draws the
                         same stream whatever the batching or world size */
  /* group payoff of a cooperator / defector in a group with N cooperators,
   * N = 0..5: (r*c*N)/5 - cost and (r*c*N)/5 (spgg.py:256-257), computed by
   * the host in the reference's order. */
  double pay_c[6];
  double pay_d[6];
  /* compact reputation (spgg_config.rep_int8): R = k*rep_unit with
   * k in [rk_min, rk_max] (int8); gain/loss per action in the same units.
   * Valid only when rep_gain_C, delta_R_D, R_min, R_max are all exact
   * multiples of a dyadic rep_unit: then every f64 sum/clip of the reference
   * is exact and the int8 path reproduces it bit for bit. */
  double rep_unit;
  int32_t rk_gain, rk_loss, rk_min, rk_max;
  double norm_rcp;    /* 1/norm_den rounded to nearest (host) */
} spgg_rep_params;

/* Device buffers, all replica-major.  n = L*L.
 *   S[2]      uint8  [n_rep][n]      S_t in S[(t-1) & 1] (iteration t reads [(t-1)&1],
 *                                    writes [t&1]).  bit0: strategy (0 = C); bits 1-4:
 *                                    bookkeeping of iteration t-1 (s_old, best
 *                                    neighbour's action matched, previous strategy,
 *                                    new state s_t)
 *   R[2]      f64    [n_rep][n]      reputation R_t in R[(t-1) & 1] (int8 R_t/rep_unit
 *                                    if rep_int8)
 *   Q         f64    [n_rep][n][2][2] q_table in the reference layout (L,L,2,2),
 *                                    updated IN PLACE: between launches it holds the
 *                                    last iteration's TD update without its NI term
 *                                    (applied by the next launch / spgg_flush).
 *                                    Double Q-learning: [n_rep][n][2][2][2] =
 *                                    q_table_1[s][a] then q_table_2[s][a] per agent
 *   pub[2]    f64    [n_rep][spgg_pub_doubles]  border records (library-internal
 *                                    layout): the Q row of the next state and
 *                                    max(0, max_diff) of every agent within M cells of
 *                                    its tile's edge, read by the neighbouring tiles
 *   md        f64    [n_rep][n]      max(0, max_diff) of the pending iteration, in place
 *                                    (kept only for replicas with kappa != 0: the NI term it
 *                                    feeds is +0 otherwise)
 *   atd       f32    [n_rep][n]      |alpha*td'| of the pending iteration (diagnostic), in place
 *                                    (likewise only for kappa != 0)
 *   draws     uint32 [slots][..][W]  the steps' random draws as BITS (INJECT/MT19937), a ring
 *                                    of spgg_draw_layout slots: iteration t uses slot
 *                                    (t-1) % slots at draws + slot*draw_slot_stride, replica
 *                                    rep at + rep*W (W = words_per_rep).  One plane per draw
 *                                    of the reference, in its order (spgg_draw_planes): plane
 *                                    2k = (rand < eps) and 2k+1 = randint(0,2) of select k
 *                                    (k = 0 the action; SARSA k = 1 next action, k = 2
 *                                    diagnostic, spgg.py:434,452); Double-Q plane 2 =
 *                                    (rand < 0.5), the table choice (algorithms.py:307).
 *                                    Agent g's bit of plane p: bit g % 32 of word
 *                                    (g / 32) * planes + p (planes interleaved per 32 agents;
 *                                    W = ceil(n/64) * 2 * planes).  INJECT: the caller writes
 *                                    slot (t-1) % slots before spgg_step(t); MT19937: the
 *                                    library's generator fills the ring
 *   mt_state  uint32 [n_rep][625]    MT19937 key[624] + pos (MT19937 only): the key before the
 *                                    run; after spgg_flush the key the reference holds after
 *                                    each replica's last executed iteration
 *   mt_snap   uint32 [snap_slots][..][625]  key snapshots (MT19937 only; library-internal:
 *                                    slot t % snap_slots = the key after iteration t),
 *                                    replica rep at + slot*mt_snap_stride + rep*625
 *   eps       f64    [n_rep][iterations+2]  eps used by iteration t
 *   stats     f64    [n_rep][stripes][iterations+2][SPGG_NSTAT]  zero-initialised;
 *                                    stripe 0 of slot t0 must hold NCOOP of S_t0 before
 *                                    stepping (stripes: spgg_stat_stripes)
 *   stop_iter int32  [n_rep]         0 while running, else the absorbing iteration
 * Initial state: S[0] = population (bits 1-7 zero), R[0] = 0, Q = initial table.
 * Final state of a replica absorbed at s: S, R in [(s-1)&1]; of a replica still
 * running after spgg_flush(t_last): S, R in [t_last&1].  Q (in place) is final
 * after spgg_flush / the absorbing launch.
 */
typedef struct {
  uint8_t* S[2];
  void* R[2];     /* double, or int8_t when spgg_config.rep_int8 */
  double* Q;
  double* pub[2];
  double* md;
  float* atd;
  uint32_t* draws;
  int64_t draw_slot_stride;   /* u32 words between draw-record ring slots (>= n_rep*words_per_rep) */
  uint32_t* mt_state;
  uint32_t* mt_snap;
  int64_t mt_snap_stride;     /* u32 words between key-snapshot slots (>= n_rep*625) */
  double* eps;
  double* stats;
  int32_t* stop_iter;
} spgg_buffers;

int spgg_abi_version(void);
/* Content hash of the sources, compiler flags and defines the library was built from
 * (build.py): the package refuses an in-tree library whose id differs from the sources. */
const char* spgg_build_id(void);
/* Number of draw planes one iteration of `algorithm` consumes: 2, 6 (SARSA), 2, 3 (Double-Q). */
int spgg_draw_planes(int32_t algorithm);
/* Detail of the context's last failure; with ctx == NULL, of the calling thread's
 * last failed spgg_create. */
const char* spgg_last_error(const spgg_ctx* ctx);

/* Environment knob read here: SPGG_APT = "1" (one agent per thread) or "max" (the
 * operator's maximum) forces the tiling; any other value fails with SPGG_E_ARG. */
int spgg_create(spgg_ctx** out, const spgg_config* cfg);
/* Copies n_rep host records to the device (stream-ordered on the null stream).  Between
 * spgg_step calls of one run a replica's kappa must not change from 0 to nonzero (the pending
 * max_diff / |alpha*td'| records of kappa == 0 replicas are not kept): a later spgg_step with
 * t0 > 1, or spgg_flush, then fails with SPGG_E_STATE (spgg_step with t0 == 1 starts a new run). */
int spgg_set_params(spgg_ctx* ctx, const spgg_rep_params* params);
int spgg_bind(spgg_ctx* ctx, const spgg_buffers* bufs);

/* Enqueue iterations t0 .. t0+n_steps-1 (1-based, as the reference's loop
 * variable i, spgg.py:368).  Replicas that reach an absorbing state stop by
 * themselves (spgg.py:405-406).  In SPGG_RNG_INJECT mode n_steps must be 1
 * and the draw planes of iteration t0 must already be in place. */
int spgg_step(spgg_ctx* ctx, int32_t t0, int32_t n_steps, void* hip_stream);

/* Apply the deferred neighbor-influence term of iteration t_last (the last
 * executed one) and its Q statistics.  Call once after the final spgg_step.
 * MT19937: also waits for the generator and restores mt_state to each replica's
 * key after its last executed iteration (the state np.random holds after the
 * reference's run).
 * SPGG_E_STATE if a replica's kappa went from 0 to nonzero since the run began
 * (its pending record was never written; see spgg_set_params). */
int spgg_flush(spgg_ctx* ctx, int32_t t_last, void* hip_stream);

/* Fill the derived history slots (SPGG_ST_SUMP / _SUMP_C / _SUMP_D of iterations 1..last,
 * SPGG_ST_SUM_WPP / _SUM_WRR / _SUM_REW_D / _SW_DC of the executed steps; last = a replica's
 * absorbing iteration, else t_last) from the counted ones.  Idempotent; enqueue it after
 * the steps whose records are read.  Replaces: the per-step np.mean calls of
 * spgg.py:383-394, 529-545 for those values. */
int spgg_history_finalize(spgg_ctx* ctx, int32_t t_last, void* hip_stream);

/* Generate the draw record of iteration t only, from mt_state (advancing it), into its
 * ring slot (MT19937 mode; for tests -- spgg_step runs the pipelined generator itself). */
int spgg_draw(spgg_ctx* ctx, int32_t t, void* hip_stream);
/* The same for iterations t0..t1 in ONE generator launch (t1 - t0 < the generator's chunk,
 * spgg_draw_layout slots / 2), as spgg_step's pipeline launches it (for tests). */
int spgg_draw_range(spgg_ctx* ctx, int32_t t0, int32_t t1, void* hip_stream);

/* Draw-record ring of INJECT / MT19937 contexts: ring slots (iterations), u32 words per
 * replica and slot, and key-snapshot slots (MT19937).  Replaces: the reference's per-step
 * np.random.rand / randint calls (algorithms.py:105-108) -- their outputs as bits. */
int spgg_draw_layout(const spgg_ctx* ctx, int32_t* slots, int64_t* words_per_rep, int32_t* snap_slots);

/* MT19937: the stream the draw generator runs on (default: one the library creates per
 * context).  Contexts of one batch may share one; call before the first spgg_step. */
int spgg_set_draw_stream(spgg_ctx* ctx, void* hip_stream);

/* P (normalised payoff, spgg.py:373-378) of every agent from S_t into
 * out[n_rep][n] (device).  Used for SPGG.P and run()'s return value. */
int spgg_payoff(spgg_ctx* ctx, int32_t t, double* out, void* hip_stream);

/* Doubles per replica of each border-record buffer (spgg_buffers.pub). */
int spgg_pub_doubles(const spgg_ctx* ctx, int64_t* per_rep);

/* History-record stripes per replica the stats buffer must hold (1 for small
 * lattices; up to 32 so that <= 64 workgroups add to one record address per
 * iteration).  Replaces: nothing (reference's per-step np.mean calls). */
int spgg_stat_stripes(const spgg_ctx* ctx, int32_t* stripes);

/* Tile shape (agents) the step kernel uses for this lattice. */
int spgg_tile_shape(const spgg_ctx* ctx, int32_t* tw, int32_t* th);

int spgg_destroy(spgg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* SPGG_ABI_H */
