/*
 * mbrl_cem.h -- C ABI of the MI355X (gfx950) MPC/CEM planning hot path.
 *
 * This is the drop-in boundary under the reference's planner API. The reference is pure
 * Python/PyTorch-CPU and has no FFI of its own; each entry point below replaces
 * one piece of the reference's Python call chain, cited per function. The Python host layer
 * (mujoco-mbrl_amd/mbrl_amd) binds these with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers (caller-owned HBM, e.g. torch tensors' data_ptr()),
 *     fp32 row-major unless stated; index buffers are int64 (torch.long).
 *   - Nothing here allocates or frees device memory, synchronises the device, or retains a pointer
 *     after it returns; scratch comes from the caller's workspace. Every call is stream-ordered on
 *     `stream` (a hipStream_t) and may be captured into a HIP graph.
 *   - Return value: MBRL_OK (0) or a negative MBRL_E* code; mbrl_last_error() then holds a
 *     thread-local message. The Python layer turns a nonzero code into RuntimeError, matching the
 *     reference's exceptions-only convention.
 *   - No HIP call happens at library load (fork safety: parallel.py:1-2,20-52 pickles planners
 *     into forkserver workers).
 */
#ifndef MBRL_CEM_H
#define MBRL_CEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MBRL_ABI_VERSION 13

typedef struct ihipStream_t* mbrl_stream_t; /* == hipStream_t */
typedef struct ihipEvent_t* mbrl_event_t;   /* == hipEvent_t  */

enum {
    MBRL_OK = 0,
    MBRL_EINVAL = -1,        /* bad argument (null pointer, non-positive size, K > N, ...) */
    MBRL_EUNSUPPORTED = -2,  /* shape outside what the kernels are built for */
    MBRL_EHIP = -3,          /* a HIP runtime call failed */
    MBRL_EWORKSPACE = -4,    /* workspace too small */
    MBRL_EPEER = -5          /* mbrl_cem_plan_sharded: another rank failed during the plan (ABI v13); this
                                rank's outputs are void, its communicator stays usable */
};

/* Cost kinds.
 * GOAL_STATE   = state_action_cost(SmoothAbsLoss, CoshLoss) on (s_{t+1}, a_t), agents.py:182-183,231.
 * MODEL_REWARD = the reward head of the dynamics model itself, evaluated at (s_{t+1}, a_t) and
 *                unnormalised: RewardAgent's compose(partial(model, ...), itemgetter(1)) cost
 *                (agents.py:342-362, models.py:143-163). Needs mbrl_mlp_shape.reward_head = 1; every
 *                step then runs the MLP twice (the state pass, then the reward pass). */
enum { MBRL_COST_GOAL_STATE = 0, MBRL_COST_MODEL_REWARD = 1 };

/* Ordering of NaN returns in elite selection. */
enum {
    MBRL_NAN_LAST = 0,  /* np.argsort(kind="stable") order: NaN after every number (CEM elites)     */
    MBRL_NAN_FIRST = 1  /* np.argmin order: the first NaN wins (RandomShootingPlanner, planners.py:184) */
};

/* Matrix-product precision of the rollout's MLP layers (mbrl_mlp_shape.precision).
 * F32   = v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation.
 * F16X3 / F16X6 = fp32 emulated on the f16 matrix cores (v_mfma_f32_16x16x32_f16, 16x the fp32
 *         matrix rate). Each operand is scaled by an exact power of two and split into P f16
 *         pieces x0 = f16(x), x1 = f16(x - x0) (, x2 = f16(x - x0 - x1)); the products x_i w_j with
 *         i + j < P accumulate in fp32.
 *         F16X3: P = 2, 3 products, operands to 22 significant bits (fp32: 24); the dropped
 *                term is 2^-22 relative.
 *         F16X6: P = 3, 6 products, operands to 33 significant bits, dropped terms <= 2^-33
 *                relative: at least fp32's operand precision with exact partial products.
 *         Operands past the split range (activations >= 2048, weights >= 128) cannot be split;
 *         a workgroup that meets one redoes its candidates in F32 (on the device, in the same
 *         call), so results never depend on the operand range. Used for goal-state costs with
 *         256 <= W <= 512; every other case runs F32. */
enum { MBRL_PRECISION_F32 = 0, MBRL_PRECISION_F16X3 = 1, MBRL_PRECISION_F16X6 = 2 };

/* Dynamics MLP shape: Linear(s+a -> W), ReLU, [Linear(W -> W), ReLU] x (L-1), Linear(W -> s).
 * models.py:96-110 (Model, L = 2) generalised to L hidden layers; E ensemble members.
 * reward_head = 1: ModelWithReward (models.py:125-141): the same trunk plus a reward head
 * Linear(W -> 1) beside the state head. */
typedef struct {
    int32_t state_dim;   /* s  (observation dim, env_wrappers.py:86 flat 'observations') */
    int32_t action_dim;  /* a */
    int32_t hidden;      /* W  (any >= 1; zero-padded inside the packed stream) */
    int32_t n_hidden;    /* L >= 1 */
    int32_t ensemble;    /* E >= 1 */
    int32_t reward_head; /* 0 or 1 */
    int32_t precision;   /* MBRL_PRECISION_* (rollout only; the packed buffer holds every weight
                            stream, so one pack serves each precision) */
} mbrl_mlp_shape;

/* Normalisation affine, TransitionsDataset.normalize_field / unnormalize_field (data.py:255-260),
 * bound as in agents.py:219-230. A zero flag = that keyword was None in the reference call. */
typedef struct {
    const float* obs_mean;  /* [s] */
    const float* obs_std;   /* [s] */
    const float* act_mean;  /* [a] */
    const float* act_std;   /* [a] */
    const float* rew_mean;  /* [1] "rewards" statistics (agents.py:340), reward_head models only */
    const float* rew_std;   /* [1] */
    int32_t normalize_state;
    int32_t unnormalize_state;
    int32_t normalize_action;
    int32_t unnormalize_reward;
} mbrl_norm;

/* Per-step cost on the (s_{t+1}, a_t) pair (planners.py:210). */
typedef struct {
    int32_t kind;             /* MBRL_COST_GOAL_STATE or MBRL_COST_MODEL_REWARD */
    int32_t has_state_cost;   /* SmoothAbsLoss term present (models.py:244-259) */
    int32_t has_action_cost;  /* CoshLoss term present (models.py:262-272) */
    int32_t _pad;
    const float* weights;     /* [s] SmoothAbsLoss.weights */
    const float* goal;        /* [s] SmoothAbsLoss.goal_state */
    float alpha_state;        /* SmoothAbsLoss.alpha (default 0.4) */
    float alpha_action;       /* CoshLoss.alpha (default 0.25) */
} mbrl_cost;

/* CEM proposal: a[t][n][d] = clip(mu[t][d] + sigma[t][d] * eps, lo, hi), eps from Philox4x32-10
 * keyed by `seed`, counter (n + n_offset, t, iteration, d >> 2). Bounds follow the reference's
 * dim-0 action bounds [max(min[0],-3), min(max[0],3)] (env_wrappers.py:52-55). */
typedef struct {
    uint64_t seed;
    int32_t iteration;
    int32_t _pad;
    const float* mu;     /* [H][a] */
    const float* sigma;  /* [H][a] */
    float lo;
    float hi;
} mbrl_sampler;

typedef struct {
    int32_t N;            /* candidates (global; == local when not sharded) */
    int32_t H;            /* horizon */
    int32_t K;            /* elites */
    int32_t iterations;   /* I */
    float alpha;          /* refit smoothing: mu <- alpha*mu + (1-alpha)*mu' */
    float lo, hi;         /* action bounds */
    float init_mu;        /* initial mean (0) */
    float init_sigma;     /* initial std ((hi-lo)/4) */
    int32_t _pad;
    uint64_t seed;
} mbrl_cem_params;

int mbrl_abi_version(void);
/* "src=<16 hex digits> arch=gfx950": the sha256 prefix of the sources the library was built from
 * (mujoco-mbrl_amd/Makefile DIGEST_FILES), so a caller can check a prebuilt library against a tree. */
const char* mbrl_build_info(void);
const char* mbrl_last_error(void);

/* ---- process-wide switches for A/B runs and for tests that force a fallback. Every option starts
 * at 0 (automatic choice); the library never reads them from the environment, so a production launch
 * cannot be redirected by a stray variable. mbrl_set_option returns the previous value, or
 * MBRL_EINVAL for an unknown option or value. Not part of any reference interface. */
enum {
    MBRL_OPT_ROLLOUT_TILE = 0,      /* fp32 rollout candidates per workgroup: 0 auto, 4, 8, 16 (16 R) */
    MBRL_OPT_SPLIT_TILE = 1,        /* F16X3 / F16X6 rollout candidates per workgroup: 0 auto, 16, 32 */
    MBRL_OPT_DEBUG_TRAJ_ABORT = 2,  /* 1: the cooperative trajectory kernel gives up at once          */
    MBRL_OPT_GD_SINGLE = 3,         /* 1: mbrl_gd_plan runs its one-workgroup kernel                  */
    MBRL_OPT_DEBUG_GD_ABORT = 4,    /* 1: the cooperative gd kernel gives up at once                  */
    MBRL_OPT_UNFUSED_UPDATE = 5,    /* 1: plans run select / refit / proposal draw as separate launches */
    MBRL_OPT_ADAM_ARITH = 6,        /* mbrl_adam_step contraction pattern: 0 = torch's; 1 + bits (test) */
    MBRL_OPT_XCD_MAP = 7,           /* 1: ensemble rollouts map workgroups member-major per XCD (A/B) */
    MBRL_OPT_TRAIN_TILE = 8,        /* training backward C tile height: 0 auto, 32, 64 (bit-identical) */
    MBRL_OPT_TRAIN_NO_FOLD = 9,     /* 1: the layer-0 weight gradient in its own launch (bit-identical) */
    MBRL_OPT_ROLLOUT_PAIR = 10,     /* column-split pairs in plans: 0 auto, 1 forced (MBRL_EUNSUPPORTED where
                                       they cannot run), 2 never; standalone rollouts never use them  */
    MBRL_OPT_SHARD_EMULATE = 11,    /* 1 (tests): mbrl_cem_plan_sharded with comm == NULL computes every
                                       other rank's shard itself in place of the all-gather (G > 1 on one GPU)
                                       and keeps each iteration's gathered costs in the workspace; 2 (timing,
                                       ABI v13): the other ranks' slots are copied from those kept costs (one
                                       launch per iteration), so the call runs exactly one rank's work: its
                                       shard's rollout, the update over all N, its own draw, the trajectory.
                                       Mode 2 is bit-identical to mode 1 after a mode-1 plan of the same
                                       problem, seed and N (any rank id); set the option before the
                                       workspace query (the kept costs live in the workspace) */
    MBRL_OPT_DEBUG_PAIR_ABORT = 12, /* 1: the column-split pair kernel gives up at once (its redo runs);
                                       2: no redo launch behind it (tests of the pair kernel's own results) */
    MBRL_OPT_TRAJ_HOP = 13,         /* cooperative trajectory hand-offs: 0 auto, 1 (P, E) grid + sc1 granules,
                                       2 per-member XCD grid + sc1, 3 XCD grid + L2-resident granules when
                                       the roll call finds the member on one XCD (A/B; same results) */
    MBRL_OPT_GD_HOP = 14,           /* the cooperative gd kernel's hand-offs, as MBRL_OPT_TRAJ_HOP             */
    MBRL_OPT_PAIR_L2 = 15,          /* column-split pair hand-offs: 0 / 1 L2-resident when both halves share an
                                       XCD (roll call), 2 always written through (A/B; same results)     */
    MBRL_OPT_TRAIN_XCD = 16,        /* training launches: 1 row bands in XCD order (A/B; same bits)           */
    MBRL_OPT_TRAIN_SPLIT = 17,      /* 1: two-hidden-layer training in the five-launch layout instead of the
                                       fused three-launch step (A/B, tests; same bits)                    */
    MBRL_OPT_DEBUG_SHARD_FAIL = 18, /* i + 1 (tests): mbrl_cem_plan_sharded reports a failed launch at
                                       iteration i on the rank MBRL_OPT_DEBUG_SHARD_FAIL_RANK names (the rank
                                       then keeps joining the all-gathers); 0 off */
    MBRL_OPT_TRAIN_FO = 19,         /* 1: the fused training step's F and O as two launches (A/B; same bits) */
    MBRL_OPT_DEBUG_SHARD_FAIL_RANK = 20, /* (tests, ABI v13) r + 1: the injected failure is rank r's only (the
                                       other ranks see it as a peer failure; under MBRL_OPT_SHARD_EMULATE a
                                       call with another rank id fails that rank's emulated slot); 0: the
                                       calling rank's, whatever its id */
    MBRL_OPT_UPDATE_SPLIT = 21,     /* (ABI v13) plans' per-iteration update as two launches that share out the
                                       elites' regeneration (select + regenerate, then refit + draw): 0 auto
                                       (K ceil(a/4) >= 2048 Philox blocks per row), 1 never, 2 always (A/B,
                                       tests; same bits) */
    MBRL_OPT_COUNT = 22
};
int mbrl_set_option(int32_t option, int32_t value);
int mbrl_get_option(int32_t option);

/* ---- multi-GPU (the reference has no distributed code): an RCCL communicator the
 * library owns. mbrl_comm_unique_id on one rank, the MBRL_COMM_ID_BYTES broadcast to the others by the
 * caller (torch.distributed), then mbrl_comm_init on every rank at once (collective), with the rank's
 * GPU current. RCCL (librccl.so.1) is opened on the first of these calls, not at load time: without it
 * they return MBRL_EUNSUPPORTED and everything else works. */
#define MBRL_COMM_ID_BYTES 128
typedef void* mbrl_comm_t;
int mbrl_comm_unique_id(void* id_out);
int mbrl_comm_init(const void* id, int32_t nranks, int32_t rank, mbrl_comm_t* comm_out);
int mbrl_comm_destroy(mbrl_comm_t comm);

/* ---- host staging: mapped, coherent pinned host memory (hipHostMalloc Mapped | Coherent) that the
 * kernels read and write directly. plan() (planners.py:14-25) takes its initial state from the host and
 * returns host tensors; passing mbrl_cem_plan a staged s0 and staged outputs replaces the two
 * host<->device copies around the plan with the plan's own first and last launches. *device_ptr is
 * the address kernels use (the same as *host_ptr under unified addressing). */
int mbrl_host_alloc(size_t bytes, void** host_ptr, void** device_ptr);
int mbrl_host_free(void* host_ptr);

/* ---- stream plumbing (no reference counterpart; ABI v12): events for ordering work between streams
 * and for the host to wait on, created without timing and without the system-scope fence a default
 * event's record ends in (which idles the GPU ~5.5 us per record). train_model's epoch loop orders its
 * row-order copies with them (mbrl_amd/models.py _OrderRing). A never-recorded event is complete. */
int mbrl_event_create(mbrl_event_t* event);
int mbrl_event_record(mbrl_event_t event, mbrl_stream_t stream);
int mbrl_stream_wait_event(mbrl_stream_t stream, mbrl_event_t event);
int mbrl_event_synchronize(mbrl_event_t event);
int mbrl_event_destroy(mbrl_event_t event);

/* ---- model upload: replaces the per-call nn.Linear weight reads of Model._forward (models.py:106-110) */
size_t mbrl_mlp_packed_bytes(const mbrl_mlp_shape* shape);
/* weights[e*NL+l] / biases[...], NL = L + 1 + reward_head: DEVICE pointers to nn.Linear weight
 * [out][in] and bias [out] (trunk layers, the state head, then the reward head), passed in a HOST
 * array. Writes the fragment-ordered weight stream the rollout kernel reads. */
int mbrl_mlp_pack(const mbrl_mlp_shape* shape, const float* const* weights, const float* const* biases,
                  void* packed, mbrl_stream_t stream);

/* ---- rollout + cost: replaces RandomShootingPlanner._generate_trajectories' model/cost loop
 * (planners.py:199-210) and DynamicsModel.forward (models.py:13-29) on its batch.
 * s0: [s] broadcast to every candidate (planners.py:204) or [N][s] when s0_per_candidate.
 * actions: [H][N][a] time-major (planners.py:200,207), or NULL to draw them from `sampler` into
 *          actions_out first (actions_out is then required).
 * costs: [E][N] per-member return sum_t cost(s_{t+1}, a_t), summed sequentially in t.
 * actions_out: [H][N][a] or NULL. states_out: [E][H][N][s] or NULL.
 * n_offset: global index of local candidate 0 (rank shard offset; keys the RNG). */
int mbrl_rollout_cost(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                      const mbrl_cost* cost, const float* s0, int32_t s0_per_candidate,
                      const float* actions, const mbrl_sampler* sampler, int32_t N, int32_t H,
                      int32_t n_offset, float* costs, float* actions_out, float* states_out,
                      mbrl_stream_t stream);

/* ---- selection: replaces np.argmin (planners.py:184) and adds CEM's stable top-K.
 * returns[n] = (sum_e costs[e][n]) / E (sequential in e; = costs[0][n] when E == 1).
 * elite_idx[0..K): the K smallest (return, index) pairs, written in ASCENDING candidate index.
 * returns_out: [N] or NULL. workspace: >= mbrl_select_workspace_bytes(N). */
size_t mbrl_select_workspace_bytes(int32_t N);
int mbrl_select_elites(const float* costs, int32_t E, int32_t N, int32_t K, int32_t nan_policy,
                       int64_t* elite_idx, float* returns_out, void* workspace, size_t ws_bytes,
                       mbrl_stream_t stream);

/* ---- CEM refit (not in the reference). Regenerates each elite's actions from
 * the counter RNG (so every rank can refit from the global elite list with no moment collective),
 * sums them in the canonical chunked order, writes mu' / sigma' ([H][a]).
 * Multi-GPU split step: SURVEY.md §8b proposed an mbrl_topk_moments (local elite moments, then an
 * all-gather of [G][2][H][a]). Here every rank runs mbrl_select_elites on the all-gathered
 * returns and mbrl_cem_refit on the global elite list: one collective per iteration instead of
 * two, and the result does not depend on the GPU count. */
size_t mbrl_refit_workspace_bytes(int32_t H, int32_t a, int32_t K);
int mbrl_cem_refit(const mbrl_sampler* sampler, int32_t H, int32_t a, const int64_t* elite_idx,
                   int32_t K, float alpha, float* mu_out, float* sigma_out, void* workspace,
                   size_t ws_bytes, mbrl_stream_t stream);

/* ---- proposal draw only (generic-callable path and RNG parity): actions_out [H][N][a]. */
int mbrl_sample_actions(const mbrl_sampler* sampler, int32_t H, int32_t a, int32_t N, int32_t n_offset,
                        float* actions_out, mbrl_stream_t stream);

/* ---- one trajectory per ensemble member: the states of a single action sequence (the final CEM
 * mean; replaces the N=1 use of planners.py:199-210). actions [H][a]; states_out [H][s] = member
 * mean; member_states_out [E][H][s] or NULL. workspace >= mbrl_trajectory_workspace_bytes. */
size_t mbrl_trajectory_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H);
int mbrl_trajectory(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const float* s0,
                    const float* actions, int32_t H, float* states_out, float* member_states_out,
                    void* workspace, size_t ws_bytes, mbrl_stream_t stream);

/* ---- whole single-GPU CEM plan: I x (rollout -> select -> refit), then the final mean's rollout.
 * mu / sigma: [H][a] final distribution. actions_out: [H][a] = clip(mu, lo, hi);
 * states_out: [H][s] rollout of actions_out (ensemble mean over members).
 * cost_hist [I][E][N], returns_hist [I][N], elite_hist [I][K]: optional per-iteration records (NULL = off).
 * rollout_events: NULL or 2*I events; pair i brackets iteration i's rollout launch on `stream`
 * (a NULL pair skips iteration i: each record leaves the GPU idle a few microseconds).
 * s0 [s] is read once, by the plan's first launch (into the workspace), and mu / sigma / actions_out /
 * states_out are written by its last launches only: all five may be device memory or mapped host
 * memory from mbrl_host_alloc (ABI v7; plan() on host tensors with no copy launch around it). */
size_t mbrl_cem_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params);
int mbrl_cem_plan(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                  const mbrl_cost* cost, const float* s0, const mbrl_cem_params* params,
                  float* mu, float* sigma, float* actions_out, float* states_out,
                  float* cost_hist, float* returns_hist, int64_t* elite_hist,
                  mbrl_event_t* rollout_events, void* workspace, size_t ws_bytes,
                  mbrl_stream_t stream);

/* ---- the same plan sharded over `nranks` GPUs, one call per rank: rank r rolls out global candidates
 * [r N / nranks, (r + 1) N / nranks) (proposals keyed by the global index), every iteration all-gathers
 * the [E][N / nranks] costs over `comm` as a step on `stream` (ncclAllGather), then every rank runs the
 * same selection over all N, the same refit and draws its own shard of the next proposals. Outputs are
 * bit-identical on every rank and to mbrl_cem_plan's for any nranks (records as mbrl_cem_plan's, over
 * all N). Replaces planners.cem_sharded_protocol's per-iteration Python loop. N % nranks == 0.
 * Every argument check runs before the first collective (the ranks pass the same shape, params and
 * nranks, so they agree on it). A launch that fails later does not end the call early: the rank skips
 * its remaining compute launches but still joins every remaining all-gather (its local costs poisoned
 * to NaN), so no peer waits on it and `comm` stays usable, and returns its own error at the end.
 * Failure is visible on every rank (ABI v13): the last iteration's all-gather also gathers one status
 * word per rank (grouped with the costs in one RCCL call), and a rank whose status word is set makes
 * every other rank return MBRL_EPEER instead of a plan over N - N / nranks candidates. With nranks > 1
 * the call therefore returns after the plan has completed on `stream` (one stream synchronisation, at
 * its end); with nranks == 1 it only enqueues, as mbrl_cem_plan.
 * comm == NULL is allowed only under MBRL_OPT_SHARD_EMULATE (tests, timing): each call then fills the
 * all-gather's rank-major buffer itself (mode 1: rolls out every rank's shard; mode 2: copies the other
 * ranks' costs kept by an earlier mode-1 plan), so one GPU runs any nranks. */
size_t mbrl_cem_plan_sharded_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params,
                                             int32_t nranks);
int mbrl_cem_plan_sharded(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                          const mbrl_cost* cost, const float* s0, const mbrl_cem_params* params, mbrl_comm_t comm,
                          int32_t nranks, int32_t rank, float* mu, float* sigma, float* actions_out,
                          float* states_out, float* cost_hist, float* returns_hist, int64_t* elite_hist,
                          mbrl_event_t* rollout_events, void* workspace, size_t ws_bytes, mbrl_stream_t stream);

/* ---- batched planning: B independent CEM plans, one per initial state s0[b] (parallel environments
 * feeding one GPU planner), in shared launches: one proposal draw, one rollout
 * of B*N candidates, one segmented selection, one batched refit per iteration. Problem b's candidate
 * n is global candidate b*N + n for the proposal RNG, so problem b's plan equals a single-problem
 * plan whose candidates are drawn with n_offset = b*N. params->N, ->K are PER problem.
 * s0: [B][s]; mu / sigma (optional): [B][H][a]; actions_out: [B][H][a] = clip(mu);
 * states_out: [B][H][s] (member mean). */
size_t mbrl_cem_plan_batch_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params, int32_t B);
int mbrl_cem_plan_batch(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                        const mbrl_cost* cost, const float* s0, int32_t B, const mbrl_cem_params* params,
                        float* mu, float* sigma, float* actions_out, float* states_out, void* workspace,
                        size_t ws_bytes, mbrl_stream_t stream);

/* ---- one CEM iteration's update after the rollout, as ONE launch (cem_update_kernel): the stable
 * top-K of the member-mean returns (as mbrl_select_elites, NAN_LAST), the refit of every row (as
 * mbrl_cem_refit) and, with next_actions, iteration sampler->iteration + 1's proposals for global
 * candidates [draw_offset, draw_offset + draw_count) drawn from the new mu / sigma (as
 * mbrl_sample_actions with n_offset = draw_offset). Bit-identical to those three calls; used by the
 * sharded (multi-GPU) plan, where every rank updates on the all-gathered costs and draws its shard.
 * costs: [E][N]; elite_idx: [K] or NULL; returns_out: [N] or NULL; mu_out / sigma_out: [H][a];
 * next_actions: [H][draw_count][a] or NULL. MBRL_EUNSUPPORTED when N > 32768 or the selection /
 * refit working set exceeds LDS: use the three calls. Not part of any reference interface. */
int mbrl_cem_update(const float* costs, int32_t E, int32_t N, int32_t K, const mbrl_sampler* sampler, int32_t H,
                    int32_t a, float alpha, int64_t* elite_idx, float* returns_out, float* mu_out, float* sigma_out,
                    float* next_actions, int32_t draw_offset, int32_t draw_count, mbrl_stream_t stream);

/* ---- gradient-descent planner: replaces GradientDescentPlanner's
 * _optimize_trajectory (planners.py:103-137) -- Adam(lr) on the action sequence through the dynamics
 * with the goal-state cost (or, for a reward_head model, the MODEL_REWARD cost of RewardAgent,
 * agents.py:336-362), stopping once mean |delta a| < stop_condition -- as one launch (forward,
 * backward and the Adam step on the device; no host round trip per iteration): Wpad/16 cooperating
 * workgroups that hand hidden vectors to each other, or one workgroup where those do not apply
 * (reward-head models, shapes outside the cooperative kernel's).
 * actions: [H][a] device, in: the initial sequence, out: the optimised one. states_out: [H+1][s]
 * = the last iteration's rollout (computed before its update, as the reference returns it).
 * iterations_out: device int32 (iterations run) or NULL. Needs ensemble == 1 and a GOAL_STATE cost
 * (reward_head == 0) or a MODEL_REWARD cost (reward_head == 1), else MBRL_EUNSUPPORTED.
 * workspace >= mbrl_gd_workspace_bytes(shape, H). */
size_t mbrl_gd_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H);
size_t mbrl_gd_batch_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H, int32_t B);
int mbrl_gd_plan(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                 const float* s0, float* actions, int32_t H, int32_t num_iterations, float stop_condition,
                 float lr, float* states_out, int32_t* iterations_out, void* workspace, size_t ws_bytes,
                 mbrl_stream_t stream);
/* B independent gradient-descent plans in shared launches (parallel environments: one start state
 * each, SURVEY.md §8f rank 3 "batching over restarts"): s0 [B][s], actions [B][H][a] (in: the initial
 * sequences, out: the optimised ones), states_out [B][H+1][s], iterations_out [B] or NULL. Each plan
 * is exactly mbrl_gd_plan's (same arithmetic, its own stop test); the cooperative grids of as many
 * plans as fit the device together run in one launch. workspace >= mbrl_gd_batch_workspace_bytes. */
int mbrl_gd_plan_batch(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                       const float* s0, float* actions, int32_t B, int32_t H, int32_t num_iterations,
                       float stop_condition, float lr, float* states_out, int32_t* iterations_out, void* workspace,
                       size_t ws_bytes, mbrl_stream_t stream);

/* ---- model training: torch.optim.Adam.step() for one fp32 parameter group
 * (torch/optim/adam.py _multi_tensor_adam, capturable = False, amsgrad = False, maximize = False),
 * the optimizer the reference's training loop steps once per batch (models.py:53-93 with the
 * optimizer of experiment.py:55-62), as one launch over all of the group's tensors. It leaves the
 * parameters, exp_avg and exp_avg_sq bit-identical to torch's own step; the caller keeps the step
 * counters (CPU tensors in torch) and computes the per-tensor scalars in double as adam.py does:
 *   step_size = float(-(lr / (1 - beta1 ** step))),  bc2_sqrt = float((1 - beta2 ** step) ** 0.5)
 * with `step` already incremented. grad is read only (weight decay does not write it back). */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    float step_size;
    float bc2_sqrt;
} mbrl_adam_tensor;

typedef struct {
    float lerp_weight;      /* float(1 - beta1) */
    float beta2;            /* float(beta2)     */
    float one_minus_beta2;  /* float(1 - beta2) */
    float eps;              /* float(eps)       */
    float weight_decay;     /* float(weight_decay); 0 = none (L2 added to the gradient, Adam not AdamW) */
} mbrl_adam_hparams;

int mbrl_adam_step(const mbrl_adam_tensor* tensors, int32_t count, const mbrl_adam_hparams* hparams,
                   mbrl_stream_t stream);

/* ---- model training: the gradient of one batch's loss for the reference's
 * MLP dynamics models -- Model (models.py:96-110: n_hidden Linear-ReLU layers and a linear state
 * head) and ModelWithReward (models.py:125-163: the same trunk, a state head and a reward head) --
 * under the loss of their train_model (models.py:53-93, 165-217): MSELoss(predicted next state,
 * next state) (+ MSELoss(predicted reward, reward)) summed over the horizon steps, i.e. what
 * `loss.backward()` leaves in each Linear's .grad after optimizer.zero_grad(). The batch is
 * `batch` transitions of the stacked dataset, rows batch_idx[0..batch) (each < transitions, not
 * checked on the device), every horizon step of each. fp32 throughout; the summation order is not
 * autograd's, so gradients match torch's to rounding, not bit for bit.
 * weight / bias: linear1 .. linear{n_hidden} (the trunk, hidden x in), linear{n_hidden+1} (state
 * head, state_dim x hidden) and, with reward_head, linear{n_hidden+2} (1 x hidden); the *_grad
 * arrays are overwritten. loss_out: 3 device floats (total, state, reward) or NULL.
 * workspace >= mbrl_train_workspace_bytes(model, batch). */
#define MBRL_TRAIN_MAX_LAYERS 10   /* n_hidden + 2 */
typedef struct {
    int32_t state_dim, action_dim, hidden, n_hidden, reward_head, horizon;
    const float* weight[MBRL_TRAIN_MAX_LAYERS];
    const float* bias[MBRL_TRAIN_MAX_LAYERS];
    float* weight_grad[MBRL_TRAIN_MAX_LAYERS];
    float* bias_grad[MBRL_TRAIN_MAX_LAYERS];
} mbrl_train_model;

typedef struct {
    const float* states;       /* [transitions][horizon][state_dim]  (TransitionsDataset.stacked) */
    const float* actions;      /* [transitions][horizon][action_dim] */
    const float* next_states;  /* [transitions][horizon][state_dim]  */
    const float* rewards;      /* [transitions][horizon], read with reward_head only */
    int64_t transitions;
} mbrl_train_data;

size_t mbrl_train_workspace_bytes(const mbrl_train_model* model, int32_t batch);
/* Byte offset in the workspace of a 32-bit status word the fused training step (two hidden layers)
 * sets bit 0 of if one of its bounded in-launch waits timed out -- a workgroup-dispatch order the
 * kernels rely on was not kept and an Adam step may have raced a read of its weights. Never expected;
 * the word is sticky (the caller reads it after training and clears it). The caller zeroes the
 * workspace once before its first use: the fused step tags its layer-0 fold partials with a serial
 * kept in the workspace. Each mbrl_train_grads / mbrl_train_epoch call clears the step's arrival
 * tickets and band counters itself (one memset on entry, ABI v13), so a step that timed out does not
 * carry stale counts into the next call. (size_t)-1 for a bad shape. */
size_t mbrl_train_status_offset(const mbrl_train_model* model, int32_t batch);
int mbrl_train_grads(const mbrl_train_model* model, const mbrl_train_data* data, const int64_t* batch_idx,
                     int32_t batch, float* loss_out, void* workspace, size_t ws_bytes, mbrl_stream_t stream);

/* A whole training epoch with Adam (models.py:63-93 with experiment.py:55-62's optimizer): for each
 * batch b = 0 .. ceil(rows / batch_size) - 1 of the device row order `order` (the last one short),
 * mbrl_train_grads on rows order[b * batch_size ..] and then mbrl_adam_step over `tensors` (one
 * parameter group: every Linear's weight and bias, grad = the model's *_grad buffers) with that
 * step's scalars step_sizes[b * count + i], bc2_sqrt[b * count + i] (host arrays, computed as for
 * mbrl_adam_step). The host issues every launch of the epoch in one call. losses: [batches][3]
 * device floats (total, state, reward per batch) or NULL. workspace as for mbrl_train_grads with
 * batch = batch_size. Two hidden layers (the reference's models): two launches per batch (forward with
 * the output layer, then the backward with the layer-0 fold) with the Adam step inside them, each
 * batch's launches also gathering the next batch's rows; the result is the per-batch calls' bit for
 * bit (tests/test_gpu_train_native.py). */
int mbrl_train_epoch(const mbrl_train_model* model, const mbrl_train_data* data, const int64_t* order, int64_t rows,
                     int32_t batch_size, const mbrl_adam_tensor* tensors, int32_t count,
                     const mbrl_adam_hparams* hparams, const float* step_sizes, const float* bc2_sqrt, float* losses,
                     void* workspace, size_t ws_bytes, mbrl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MBRL_CEM_H */
