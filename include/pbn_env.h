/*
 * pbn_env.h -- C-ABI of the MI355X batched PBN environment step (libpbn_env.so).
 *
 * This is the drop-in boundary for the gym-PBN state-transition hot path that
 * jakub-zarzycki2022/pbn-rl drives.  The reference binds no native code: it
 * calls the external Python package gym_PBN (requirements.txt:11,
 * gym-PBN[vis]==1.1.1 + an unpublished fork) through gymnasium:
 *
 *   gym.make("gym-PBN/PBNEnv", N=, genes=, logic_functions=[, min_attractors=])
 *        train_assa_BQN.py:121-124, model_tester.py:409-413     -> pbn_net_create
 *   env.reset() -> ((state, target), info)
 *        bdq_model/__init__.py:161,204                         -> pbn_reset
 *   env.step(actions) -> (obs, reward, terminated, truncated, info)
 *        bdq_model/__init__.py:177, graph_classifier/__init__.py:148,
 *        model_tester.py:561,624, ddqn_per/__init__.py:354     -> pbn_step
 *   env.close()  train_BDQ.py:116                              -> pbn_net_destroy
 *   T frames of the frame loop bdq_model/__init__.py:172-213     -> pbn_rollout
 *   compute_ssd_hist(env, model, resets, iters) train_pbn_28.py:257 -> pbn_rollout + pbn_state_histogram
 *   BranchingDQN.predict + list(action.unique())
 *        bdq_model/__init__.py:69-98,176                       -> pbn_bilinear_targets (first layer),
 *                                                                 pbn_qnet_heads (the other layers),
 *                                                                 pbn_heads_to_flipmask / pbn_q_to_flipmask,
 *                                                                 or pbn_qnet_flipmask (both in one)
 *   update_policy's np.stack of sampled Transitions
 *        bdq_model/__init__.py:100-109                         -> pbn_obs_unpack, pbn_replay_batch
 *   update_policy (forwards, TD loss, backward, clamp, Adam)
 *        bdq_model/__init__.py:100-139                         -> pbn_bdq_learn (+ pbn_bdq_layout,
 *                                                                 pbn_bdq_pack, pbn_replay_store,
 *                                                                 pbn_replay_advance)
 *   a frame loop captured once and replayed (no reference counterpart)
 *                                                              -> pbn_step_dev, pbn_q_to_flipmask_dev
 *   the hand-off of a rollout's transitions to the learner (north_star's per-rollout gather;
 *   at world 1 the learner's own shard into its receive slot)  -> pbn_copy_async
 *
 * The Python facade (pbn_rl_amd.env.PBNEnv / pbn_rl_amd.vector_env.VectorPBNEnv)
 * keeps that gym surface and calls these entry points through ctypes;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every entry point returns 0 or a negative PBN_E* code; pbn_last_error()
 *     returns a thread-local message for the last failure on the calling thread;
 *   - the caller owns every device buffer (plain device pointers, e.g. from
 *     torch tensors); a pbn_net owns only its device-resident tables;
 *   - calls are asynchronous on the caller's HIP stream (hipStream_t passed as
 *     void*; NULL = the default stream); no entry point synchronises, allocates
 *     or frees inside pbn_reset/pbn_step, so both can be captured in a hipGraph;
 *   - a pbn_net is bound to the device that was current at create time and is
 *     not thread-safe: use one per GPU / process;
 *   - envs are processed in groups of 32 consecutive envs (bit-sliced layout):
 *     n_envs and env_offset must be multiples of 32, except that pbn_reset and
 *     pbn_step take any n_envs (ABI 9: the last group is partial; its missing
 *     envs are neither read nor written, and the others' results do not depend on
 *     them: the scalar gym facade steps n_envs = 1).  Randomness depends only
 *     on (seed, global env id = env_offset + local id, step), so sharding envs
 *     across GPUs gives bit-identical results.
 *
 * Device data layout for n envs with W = ceil(n_nodes / 32) state words:
 *   state, flipmask          uint32 [W][n]   (SoA word planes; bit i of word w = node 32w+i)
 *   target                   uint8  [n]      (attractor id; 0xFF = none)
 *   t                        uint8  [n]      (steps taken in the current episode)
 *   reward                   float  [n]
 *   flags                    uint8  [n]      (PBN_FLAG_* bits)
 *
 * Step semantics: DESIGN.md "Step semantics" (frozen; gym_PBN is unavailable).
 */
#ifndef PBN_ENV_H
#define PBN_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBN_ABI_VERSION 11

#define PBN_MAX_NODES 128
#define PBN_MAX_ARITY 4
#define PBN_MAX_FUNCS_PER_NODE 16
#define PBN_MAX_ATTRACTORS 254
#define PBN_MAX_GATES 224          /* and 32 * ceil(n_nodes / 32) + n_gates <= 256 */
#define PBN_MAX_SETTLE 4096        /* cap of settle_max (synchronous updates per env step) */
#define PBN_NO_TARGET 0xFF

/* error codes */
#define PBN_OK 0
#define PBN_EINVAL (-22)
#define PBN_ENOMEM (-12)
#define PBN_EDEVICE (-5)

/* pbn_step mode bits */
#define PBN_MODE_AUTORESET 1u      /* done envs restart: state_out/target/t hold the new episode */
#define PBN_MODE_RANDOM_ACTIONS 2u /* actions drawn in-kernel (3 uniform ints in [0,N], 0 = no-op,
                                      bdq_model/__init__.py:76); flipmask is an OUTPUT */

/* flags bits */
#define PBN_FLAG_TERMINATED 1u     /* s' is a state of the env's target attractor */
#define PBN_FLAG_TRUNCATED 2u      /* t' == horizon */
#define PBN_FLAG_IN_ATTRACTOR 4u   /* s' is a state of some attractor */
#define PBN_FLAG_PERTURBED 8u      /* a perturbation fired this step */
#define PBN_FLAG_RESET 16u         /* autoreset happened: state_out is a fresh start */
#define PBN_FLAG_UNSETTLED 32u     /* settle law: settle_max updates ran and s' is in no attractor */

/*
 * Network description (semantic form; the library derives its kernel encodings).
 * Function f of node i (node_func_start[i] <= f < node_func_start[i+1]) has
 * func_arity[f] <= 4 inputs func_inputs[4f..4f+arity) (plane references, below) and truth
 * table func_table[f]: bit m = value when input j = bit j of m.
 * func_threshold[f] is the cumulative selection threshold c_f in units of
 * 2^-prob_bits (strictly: c_{f-1} <= c_f, last of a node == 2^prob_bits).
 * perturb_cdf[m-1] = floor(2^32 * (1 - (1-p)^m)), m = 1..n_nodes.
 * Attractor a owns states attractor_start[a] .. attractor_start[a+1]-1; state k
 * is words attractor_states[k*W .. k*W+W).  reward_table[(2*term + wrong)*(N+1) + k]
 * with k = popcount(flipmask), wrong = in some non-target attractor.
 *
 * Step law (settle_max).  0 or 1: one synchronous update per env step (DESIGN.md "Step
 * semantics").  K >= 2, the settle law: after the intervention the network keeps updating
 * synchronously until the state is a state of some attractor, at most K updates in all;
 * flags carry PBN_FLAG_UNSETTLED when the K-th update still left it outside every attractor.
 * That is the "intervene, then run to a (pseudo-)attractor" step that the reference's
 * recorded bb33 evaluation pins (data/results/pbn_33_3.pkl under model_tester.py:587-658;
 * DESIGN.md "Parity status").  Update 0 draws its actions, autoreset and perturbation from the
 * one-update law's ENV / PERT calls, updates k >= 1 their perturbation from SETTLE_ENV; every
 * update's rule selection (k >= 0) is keyed per env (ABI 7): node i's uniform is the top
 * prob_bits bits of 16-bit field i & 1 of word (i >> 1) & 3 of SETTLE_SEL call (k << 8 | i >> 3)
 * of (env, step) -- so every env runs its own sequence of updates (DESIGN.md "Step law").
 */
typedef struct pbn_net_desc {
  int32_t n_nodes;
  int32_t n_funcs;
  int32_t prob_bits;     /* 4, 8, 12 or 16 */
  int32_t horizon;       /* 0 = no truncation, else 1..255 */
  const int32_t* node_func_start;   /* [n_nodes + 1] */
  const int32_t* func_arity;        /* [n_funcs] */
  const int32_t* func_inputs;       /* [n_funcs * 4], unused slots -1 */
  const uint32_t* func_table;       /* [n_funcs] */
  const uint32_t* func_threshold;   /* [n_funcs] */
  const uint32_t* perturb_cdf;      /* [n_nodes] */
  int32_t n_attractors;             /* 0..254 */
  int32_t n_attractor_states;
  const int32_t* attractor_start;   /* [n_attractors + 1] */
  const uint32_t* attractor_states; /* [n_attractor_states * W] */
  const float* reward_table;        /* [4 * (n_nodes + 1)] */
  /* Combinational gates: functions of more than 4 inputs, lowered by the compiler
   * (pbn_rl_amd/lowering.py) into functions of at most 4 "planes".  A plane reference
   * r < n_nodes is node r of the pre-step state s1; r >= n_nodes is gate r - n_nodes.  Gate g
   * may read nodes and gates < g; func_inputs may hold any reference.  All gates are evaluated
   * on s1, like the node functions, so the update stays synchronous.  0 gates = none. */
  int32_t n_gates;
  const int32_t* gate_arity;        /* [n_gates] 0..4 */
  const int32_t* gate_inputs;       /* [n_gates * 4], unused slots -1 */
  const uint32_t* gate_table;       /* [n_gates] */
  int32_t settle_max;               /* 0..PBN_MAX_SETTLE, see "Step law" above (ABI 3) */
} pbn_net_desc;

typedef struct pbn_net pbn_net;

/* Compile + upload the tables to the current device. */
int pbn_net_create(const pbn_net_desc* desc, pbn_net** out);
int pbn_net_destroy(pbn_net* net);
/* W = state words per env. */
int pbn_net_words(const pbn_net* net);

/*
 * Start episodes for envs [env_offset, env_offset + n_envs): state uniform over
 * the states of a uniformly drawn attractor, target a different attractor
 * (or a uniform random state and PBN_NO_TARGET when there are no attractors),
 * t = 0.  Draws are keyed by (seed, global env id, step).
 */
int pbn_reset(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
              uint32_t* d_state, uint8_t* d_target, uint8_t* d_t, void* stream);

/*
 * One env step of every env (the hot path): one synchronous PBN transition, or under the
 * settle law (settle_max >= 2) the intervention followed by updates until an attractor.
 *   d_state        in   [W][n]  current observation s
 *   d_flipmask     in   [W][n]  intervention flips (bit a-1 for action a > 0);
 *                  out  with PBN_MODE_RANDOM_ACTIONS (the actions drawn)
 *   d_target       in/out [n]   rewritten only for envs that autoreset
 *   d_t            in/out [n]
 *   d_state_out    out  [W][n]  next observation (reset state for autoreset envs)
 *   d_final_state  out  [W][n]  s' (the transition result) -- may be NULL
 *   d_reward, d_flags  out [n]
 * d_state_out must not alias d_state.
 */
int pbn_step(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
             uint32_t mode, const uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
             uint8_t* d_t, uint32_t* d_state_out, uint32_t* d_final_state, float* d_reward,
             uint8_t* d_flags, void* stream);

/*
 * pbn_step with the step index read from device memory (*d_step, 8-byte aligned) when the
 * kernel runs instead of passed by value, so one captured hipGraph of a frame (act + step +
 * replay + update) can be replayed for successive steps: the caller advances *d_step on the
 * stream (e.g. a captured add).  Results are bit-identical to pbn_step(step = *d_step).
 */
int pbn_step_dev(pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset, int64_t n_envs,
                 uint32_t mode, const uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                 uint8_t* d_t, uint32_t* d_state_out, uint32_t* d_final_state, float* d_reward,
                 uint8_t* d_flags, void* stream);

/*
 * pbn_step_dev_store (ABI 11): pbn_step_dev that also writes the step's transitions into a replay
 * ring, the layout pbn_replay_store writes (replaces the learning frame's separate ring-store
 * launch, pbn_rl_amd/replay.py BDQLearner's captured frame).  One-update law only (settle_max < 2;
 * PBN_EINVAL otherwise).  d_state is updated in place.  Env e's row is (*d_pos + e) mod capacity
 * (d_pos read when the kernel runs; not advanced): state = s as the step read it (bits past N
 * cleared), next_state = s' before an autoreset (= d_final_state), target = the target before
 * the step, action = d_actions_in's n_branches int32 of env e, reward, done = (flags & done_mask)
 * != 0 (done_mask 0: flags != 0), also into d_done_out[e] when not null.
 */
typedef struct pbn_ring_store {
  int64_t capacity;            /* >= n_envs */
  const int64_t* d_pos;
  uint32_t* d_state;           /* [W][capacity] */
  uint32_t* d_next_state;      /* [W][capacity] */
  uint8_t* d_target;           /* [capacity] */
  int32_t* d_action;           /* [capacity][n_branches] */
  float* d_reward;             /* [capacity] */
  uint8_t* d_done;             /* [capacity] */
  const int32_t* d_actions_in; /* [n_envs][n_branches] */
  int32_t n_branches;          /* 1..8 */
  uint32_t done_mask;
  uint8_t* d_done_out;         /* nullable: [n_envs] */
} pbn_ring_store;

int pbn_step_dev_store(pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset, int64_t n_envs,
                       uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target, uint8_t* d_t,
                       uint32_t* d_final_state, float* d_reward, uint8_t* d_flags, const pbn_ring_store* ring,
                       void* stream);

/*
 * n_steps synchronous transitions in one launch (steps step .. step+n_steps-1), with the
 * envs' state kept on chip between steps.  Bit-identical to n_steps successive pbn_step
 * calls that ping-pong d_state.  State, target and t are updated in place.
 *   d_flipmask     [n_steps][W][n]  in, or out with PBN_MODE_RANDOM_ACTIONS
 *   d_obs          [n_steps][W][n]  out: observation before each step (nullable)
 *   d_final_state  [n_steps][W][n]  out: s' of each step (nullable)
 *   d_reward, d_flags  [n_steps][n] out
 */
int pbn_rollout(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                void* stream);

/*
 * pbn_rollout with one more output (ABI 4):
 *   d_updates  [n_steps][n] uint16 out (nullable): the synchronous updates applied in each
 *              env-step, 1 under the one-update law, 1..settle_max under the settle law (the
 *              settle length; the env-step carries PBN_FLAG_UNSETTLED when it reached settle_max
 *              outside every attractor).
 * Under the settle law the pipelined kernel runs one update per iteration for every env on its
 * own plan (the selection keyed per env): an env starts its next step as soon as its current
 * step ends, whatever the other envs of its 32-env word do.
 *   the frame loop bdq_model/__init__.py:172-213 on the env constructed at train_BDQ.py:50 /
 *   model_tester.py:409-413, whose step runs to an attractor (model_tester.py:616-626)
 */
int pbn_rollout_ex(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                   int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                   uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                   uint16_t* d_updates, void* stream);

/*
 * pbn_rollout_ex with a copy riding along (ABI 8): the launch also copies copy_bytes from
 * d_copy_src to d_copy_dst (16-byte aligned, non-overlapping, neither one of this launch's
 * buffers).  The copy is complete when the launch is, on the same stream.  The pipelined
 * one-update kernel runs with a fourth wave per block that moves the block's share of the copy,
 * paced by the block's step barriers (up to four 16-byte vectors per lane and step, else in one
 * burst), and exits; the settle kernel and the wave kernel get pbn_copy_async right after the
 * launch, as does a launch of no steps.  The world-1 hand-off uses it to move rollout k's records into the learner's
 * receive slot during rollout k + 1 (pbn_rl_amd/distributed.py ShardedRollout.gather): the
 * receive half of the gather's point-to-point exchange, for the learner's own shard.
 */
int pbn_rollout_copy(pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                     int32_t n_steps, uint32_t mode, uint32_t* d_state, uint32_t* d_flipmask, uint8_t* d_target,
                     uint8_t* d_t, uint32_t* d_obs, uint32_t* d_final_state, float* d_reward, uint8_t* d_flags,
                     uint16_t* d_updates, void* d_copy_dst, const void* d_copy_src, int64_t copy_bytes,
                     void* stream);

/*
 * State histogram, the accumulation step of the steady-state distribution
 * (gym_PBN.utils.eval.compute_ssd_hist, train_pbn_28.py:257, train_pbn_10.py:257):
 * d_hist[d_states[r * row_stride + c] & (2^n_bits - 1)] += 1 for r < n_rows, c < n_cols.
 * Uses word 0 of each state (networks with n_nodes <= 32: pass the [steps][1][n] obs or
 * final_state output of pbn_rollout with row_stride = n).  1 <= n_bits <= 32; 32-bit counters;
 * the caller zeroes d_hist (2^n_bits entries).
 */
int pbn_state_histogram(const uint32_t* d_states, int64_t n_rows, int64_t n_cols, int64_t row_stride,
                        int32_t n_bits, uint32_t* d_hist, void* stream);

/*
 * Agent edges of the batched BDQ frame loop (bdq_model/__init__.py:69-98,172-177;
 * SURVEY.md 8(d) config 5).  The Q-network forward itself runs in PyTorch between them.
 *
 * pbn_obs_unpack replaces the host np.stack((state, target)) -> float tensor of
 * BranchingDQN.predict (bdq_model/__init__.py:92-93) for a whole batch:
 *   d_obs  out  float [2][n][N]: [0][e][i] = bit i of env e's state, [1][e][i] = bit i of
 *               the first state of env e's target attractor (0 without a target)
 *               -- the (2, B, N) input of BranchingQNetwork (bdq_model/network.py:55-57).
 * n_envs multiple of 32, n_envs * n_nodes < 2^31, d_obs 16-byte aligned.
 */
int pbn_obs_unpack(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                   float* d_obs, void* stream);

/*
 * The bilinear first layer of BranchingQNetwork (bdq_model/network.py:8-21) for the
 * observation pbn_obs_unpack would build, straight from the packed state:
 *   d_y[e][o] = d_bias[o] + sum over the set bits i of env e's state of d_T[target_e][i][o]
 *   d_T     in   float [n_attr][n_nodes][out_dim]: T[a][i][o] = sum_j t_a[j] W[o][i][j], t_a the
 *                first state of attractor a (the caller's GEMM; W = the layer's weight)
 *   d_bias  in   float [out_dim];  d_y out float [n][out_dim]
 * Envs without a target (id >= n_attr) get the bias.  n_envs multiple of 32, out_dim a
 * multiple of 4 in 4..1024, d_T / d_bias / d_y 16-byte aligned.
 * Rows are added in ascending i (fp32; not bit-identical to a GEMM's order).  leaky != 0 applies
 * the network's LeakyReLU (x > 0 ? x : x * slope) before the store.
 */
int pbn_bilinear_targets(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                         const float* d_T, const float* d_bias, int32_t out_dim, int32_t leaky, float slope,
                         float* d_y, void* stream);

/*
 * pbn_q_to_flipmask replaces epsilon-greedy predict + list(action.unique()) + the env's
 * action decoding (bdq_model/__init__.py:69-98,176; action a > 0 flips node a-1, :81-84):
 *   d_q         in   float [n][n_branches][n_actions], n_actions == n_nodes + 1, 16-byte aligned
 *   epsilon     explore with probability epsilon: env e explores iff EXPLORE word 0 <
 *               floor(epsilon * 2^32); its branch k action is then
 *               (word (k + 1) * (N+1)) >> 32, words numbered across EXPLORE calls 0, 1
 *               (uniform over [0, N] to (N+1)/2^32, as np.random.randint at :76);
 *               otherwise argmax over the branch (first
 *               maximum, NaN counts as the maximum: torch.argmax at :96).  EXPLORE = Philox
 *               stream 4 keyed by (seed, global env id, step), as in DESIGN.md.
 *   d_flipmask  out  uint32 [W][n]: bit a-1 set for every distinct action a > 0
 *   d_actions   out  int32 [n][n_branches] (nullable): the chosen actions
 * n_branches 1..7.  n_envs and env_offset multiples of 32.
 */
int pbn_q_to_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, uint64_t env_offset, int64_t n_envs,
                      int32_t n_branches, int32_t n_actions, const float* d_q, float epsilon,
                      uint32_t* d_flipmask, int32_t* d_actions, void* stream);

/*
 * pbn_q_to_flipmask with the step index read from device memory, as pbn_step_dev, and
 * epsilon read from *d_epsilon when that is not NULL (clamped to [0, 1], NaN -> 0), so an
 * epsilon schedule can advance on the device between graph replays.
 */
int pbn_q_to_flipmask_dev(const pbn_net* net, uint64_t seed, const uint64_t* d_step, uint64_t env_offset,
                          int64_t n_envs, int32_t n_branches, int32_t n_actions, const float* d_q,
                          float epsilon, const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions,
                          void* stream);

/*
 * pbn_q_to_flipmask on the raw head outputs of BranchingQNetwork instead of Q:
 *   d_heads  in  float [n_branches + 1][n][n_actions], head 0 = the value head (output 0 used),
 *                heads 1.. = the advantage heads (bdq_model/network.py:55-61)
 * The dueling combination is done in the kernel: q_a = (v + adv_a) - mean with mean the
 * sequential sum of adv over a divided by n_actions, then as pbn_q_to_flipmask.  d_step and
 * d_epsilon are optional device pointers (NULL: use step / epsilon), as in the _dev forms.
 */
int pbn_heads_to_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step,
                          uint64_t env_offset, int64_t n_envs, int32_t n_branches, int32_t n_actions,
                          const float* d_heads, float epsilon, const float* d_epsilon, uint32_t* d_flipmask,
                          int32_t* d_actions, void* stream);

/*
 * The layers of BranchingQNetwork after the bilinear one (bdq_model/network.py:35-61), fused
 * into one MFMA kernel (v_mfma_f32_32x32x2_f32, exact f32 k-ordered fmaf chains):
 *   d_y     in   float [n][256]: the bilinear layer after its LeakyReLU (pbn_bilinear_targets
 *                with leaky != 0)
 *   d_w1 [128][256], d_b1 [128]; d_w2 [64][128], d_b2 [64]; d_w3 [32][64], d_b3 [32]: the trunk
 *                Linear layers (torch's (out, in) layout), each followed by LeakyReLU(slope)
 *   d_wh1 [64 H][32], d_bh1 [64 H]: the H = n_heads first head layers stacked (value head
 *                first), each followed by LeakyReLU; d_wh2 [H][A][64], d_bh2 [H][A]: the
 *                second head layers (the value head zero-padded to A outputs)
 *   d_heads out  float [H][n][A]: the raw head outputs pbn_heads_to_flipmask consumes
 * n_envs a multiple of 32; n_heads 1..8; n_actions (A) 1..128; d_y and the weight matrices
 * 16-byte aligned.  Summation order differs from a GEMM library's: compare with a tolerance.
 */
int pbn_qnet_heads(const pbn_net* net, int64_t n_envs, const float* d_y, const float* d_w1, const float* d_b1,
                   const float* d_w2, const float* d_b2, const float* d_w3, const float* d_b3, const float* d_wh1,
                   const float* d_bh1, const float* d_wh2, const float* d_bh2, int32_t n_heads, int32_t n_actions,
                   float slope, float* d_heads, void* stream);

/*
 * pbn_qnet_heads and pbn_heads_to_flipmask in one launch: the same layers, then, per env, the
 * dueling combination, epsilon-greedy and flip masks exactly as pbn_heads_to_flipmask computes
 * them (same q_a order, same EXPLORE draws), without the (K+1, n, A) head outputs in HBM.
 * Arguments as those two functions (n_branches = K, the heads are K + 1; n_actions = N + 1);
 * d_step / d_epsilon, when non-null, are read when the kernel runs (graph replays).
 *   bdq_model/__init__.py:69-98,176 (predict + list(action.unique())) after the bilinear layer
 */
int pbn_qnet_flipmask(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step, uint64_t env_offset,
                      int64_t n_envs, const float* d_y, const float* d_w1, const float* d_b1, const float* d_w2,
                      const float* d_b2, const float* d_w3, const float* d_b3, const float* d_wh1, const float* d_bh1,
                      const float* d_wh2, const float* d_bh2, int32_t n_branches, int32_t n_actions, float slope,
                      float epsilon, const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions,
                      void* stream);

/*
 * pbn_qnet_heads / pbn_qnet_flipmask with the bilinear layer (+ LeakyReLU) computed in the same
 * launch from the packed state, in place of d_y: the arguments of pbn_bilinear_targets (d_state,
 * d_target, d_T, d_b0 = the layer's bias [256], out_dim 256) followed by those of the function
 * it extends.  d_T here is pbn_bilinear_targets' table with every 256-output row stored as 16 x 16
 * transposed (ABI 5): float [n_attr][n_nodes][16][16], element [a][i][j][q] = T[a][i][16 q + j]
 * (a lane's 16 MFMA operands of one node are contiguous); d_T and d_b0 16-byte aligned.  The
 * envs are sorted by target within domains of 1,024 (each block takes its 128-env slice of its
 * domain's order), so a wave's 16 envs mostly share one target's table, and the layer runs on the
 * MFMAs (k = node, 0/1 state bits as the B operand);
 * its sums are exact f32 but grouped differently from pbn_bilinear_targets' sequential adds:
 * compare with a tolerance.  This is config 5's acting frame in one launch before pbn_step.
 */
int pbn_qnet_heads_from_state(const pbn_net* net, int64_t n_envs, const uint32_t* d_state, const uint8_t* d_target,
                              const float* d_T, const float* d_b0, const float* d_w1, const float* d_b1,
                              const float* d_w2, const float* d_b2, const float* d_w3, const float* d_b3,
                              const float* d_wh1, const float* d_bh1, const float* d_wh2, const float* d_bh2,
                              int32_t n_heads, int32_t n_actions, float slope, float* d_heads, void* stream);
int pbn_qnet_flipmask_from_state(const pbn_net* net, uint64_t seed, uint64_t step, const uint64_t* d_step,
                                 uint64_t env_offset, int64_t n_envs, const uint32_t* d_state,
                                 const uint8_t* d_target, const float* d_T, const float* d_b0, const float* d_w1,
                                 const float* d_b1, const float* d_w2, const float* d_b2, const float* d_w3,
                                 const float* d_b3, const float* d_wh1, const float* d_bh1, const float* d_wh2,
                                 const float* d_bh2, int32_t n_branches, int32_t n_actions, float slope,
                                 float epsilon, const float* d_epsilon, uint32_t* d_flipmask, int32_t* d_actions,
                                 void* stream);

/*
 * n transitions into the learner's replay ring (pbn_rl_amd/replay.py DeviceReplay), in one launch:
 * env e's state / next_state (uint32 [words][n]), target (uint8 [n]), action (int32 [n][n_branches]),
 * reward (float [n]) and done (uint8 [n], nonzero = done) go to slot (*d_pos + e) mod capacity of
 * the ring arrays (state / next_state uint32 [words][capacity], target uint8 [capacity], action
 * int32 [capacity][n_branches], reward float [capacity], done uint8 [capacity] as 0/1).  d_pos
 * (int64, device memory) is read, not advanced.  capacity >= n.  With done_mask != 0, d_done is the
 * env's flags and done = (flags & done_mask) != 0 (PBN_FLAG_TERMINATED | PBN_FLAG_TRUNCATED: the
 * frame's done); d_done_out (optional, uint8 [n]) receives the same 0/1.  The optional pairs
 * d_state_dst / d_state_src (uint32 [words][n]) and d_target_dst / d_target_src (uint8 [n]) are
 * element copies done in the same pass after each element of d_state / d_target is read (a
 * destination may be d_state / d_target itself): a captured frame's copy of the stepped state back
 * into the env and its carried pre-step target, without launches of their own.
 */
int pbn_replay_store(int64_t n, const int64_t* d_pos, int64_t capacity, int32_t words, int32_t n_branches,
                     const uint32_t* d_state, const uint32_t* d_next_state, const uint8_t* d_target,
                     const int32_t* d_action, const float* d_reward, const uint8_t* d_done, uint32_t done_mask,
                     uint8_t* d_done_out, uint32_t* d_ring_state, uint32_t* d_ring_next_state, uint8_t* d_ring_target,
                     int32_t* d_ring_action, float* d_ring_reward, uint8_t* d_ring_done, uint32_t* d_state_dst,
                     const uint32_t* d_state_src, uint8_t* d_target_dst, const uint8_t* d_target_src, void* stream);

/*
 * A captured learning frame's counters and the update's rows, one single-block launch (no
 * reference counterpart: the reference keeps these on the host).  All int64 / double / float
 * one-element device tensors; each optional one is skipped when null:
 *   n_store > 0   *d_pos = (*d_pos + n_store) mod capacity, *d_size = min(*d_size + n_store, capacity)
 *   d_step        += 1 (the env step index of the next frame)
 *   d_eps64       = max(eps_final, *d_eps64 - eps_step) (decrement_epsilon, bdq_model/__init__.py:141-148);
 *                   d_eps32 its fp32 copy
 *   n_idx > 0     d_idx int64 [n_idx]: rows uniform over [0, *d_size) with replacement (row b of draw
 *                 c = *d_counter: mulhi64 of the REPLAY Philox pair of (seed, b, c) and the size);
 *                 *d_counter then advances by 1
 */
int pbn_replay_advance(int64_t n_store, int64_t capacity, int64_t* d_pos, int64_t* d_size, int64_t* d_step,
                       double* d_eps64, float* d_eps32, double eps_final, double eps_step, int64_t n_idx,
                       uint64_t seed, int64_t* d_counter, int64_t* d_idx, void* stream);

/*
 * One replay batch for the learner's update (pbn_rl_amd/replay.py DeviceReplay), in one launch:
 * rows d_idx[0..batch) (int64, < capacity) of the ring -- d_state / d_next_state uint32 [W][capacity],
 * d_target uint8 [capacity], d_action int32 [capacity][n_branches], d_reward float [capacity],
 * d_done uint8 [capacity] -- into
 *   d_x       float [2][2 batch][N]: plane 0 = the states (rows 0..batch-1) and next states
 *             (rows batch..2 batch-1) as 0/1, plane 1 = the first state of each row's target
 *             attractor (zeros without one), i.e. pbn_obs_unpack of both, concatenated by rows
 *   d_actions int64 [batch][n_branches], d_rewards float [batch], d_masks float [batch] (= done)
 */
int pbn_replay_batch(const pbn_net* net, int64_t batch, const int64_t* d_idx, int64_t capacity,
                     const uint32_t* d_state, const uint32_t* d_next_state, const uint8_t* d_target,
                     const int32_t* d_action, int32_t n_branches, const float* d_reward, const uint8_t* d_done,
                     float* d_x, int64_t* d_actions, float* d_rewards, float* d_masks, void* stream);

/*
 * The learner's TD loss on raw head outputs (bdq_model/__init__.py:111-126; pbn_rl_amd/replay.py
 * bdq_update), and its gradient, in one launch:
 *   d_online  in   float [K+1][2B][A]: the online network's raw head outputs (head 0 = value,
 *                  output 0) for the batch's states (rows 0..B-1) and next states (rows B..2B-1)
 *   d_target  in   float [K+1][B][A]: the target network's raw head outputs for the next states
 *   d_actions in   int64 [B][K], d_rewards float [B], d_masks float [B]
 *   d_loss    out  float [1]: mean over (b, k) of (r_b + q_T(b, k, a*) gamma m_b - q(b, k, a_bk))^2,
 *                  q = (v + adv_a) - mean(adv) (the dueling), a* = argmax_a q(B + b, k, a) (first
 *                  maximum, NaN maximal)
 *   d_grad    out  float [K+1][2B][A]: d loss / d d_online (0 for rows B.. and the value head's
 *                  outputs past 0)
 *   d_scratch      float [ceil(B / 8)]: per-block partial sums of the loss
 * batch = B, n_branches = K (1..7), n_actions = A (1..128).  fp32; the dueling means are
 * sequential sums, so the values equal PyTorch's to rounding.  Two launches (the pass over the
 * rows, then the partial sums added in order).
 */
int pbn_bdq_td_loss(const float* d_online, const float* d_target, const int64_t* d_actions, const float* d_rewards,
                    const float* d_masks, int32_t batch, int32_t n_branches, int32_t n_actions, float gamma,
                    float* d_loss, float* d_grad, float* d_scratch, void* stream);

/*
 * The whole update_policy step (bdq_model/__init__.py:100-139) on a flat parameter buffer, for the
 * reference's network BranchingQNetwork((N, N), N + 1, K) (bdq_model/network.py:24-63: bilinear
 * N x N -> 256, trunk 256-128-64-32, K + 1 heads 32-64-(N+1), LeakyReLU).  Replaces the sampled
 * batch's np.stack and upload (:102-109), both forwards, the target, the MSE, the backward, the
 * per-tensor gradient clamp (:129-130) and optimizer.step() (:131): three launches.
 *
 * pbn_bdq_layout: offsets[0..11] (floats, 16-float aligned) of the segments bilinear weight
 *   (256, N, N), bilinear bias (256), the trunk's three weight (out, in) / bias pairs, the heads'
 *   first layers (K+1, 64, 32) and biases (K+1, 64), second layers (K+1, N+1, 64) and biases
 *   (K+1, N+1) -- head 0 is the value head, whose rows / biases past output 0 are zero padding;
 *   offsets[12] = the total.  Parameters, Adam's moments and d_grad share this layout.
 * pbn_bdq_learn_workspace: bytes of the update's workspace at batch B (a multiple of 16).
 * pbn_bdq_image_floats (ABI 10): floats of a network's image, the d_Tq / d_target_Tq buffers.
 * pbn_bdq_pack: the image of the weights d_params into d_Tq: first the bilinear layer contracted
 *   with each attractor's first state, T[t][i][o] = sum_j x_t[j] W[o][i][j], stored
 *   [t][i][j][q] = T[t][i][16 q + j] (the table pbn_qnet_*_from_state read, n_attr * N * 256
 *   floats); then (ABI 10) the dense layers' weights as 16 x 16 tiles in the update kernels'
 *   MFMA-fragment orders (pbn_learn.hip make_image).  Needed once per parameter version not
 *   written by pbn_bdq_learn (initial weights, a loaded checkpoint, the target network after a
 *   soft update).
 * pbn_bdq_learn: rows d_idx [B] of the replay ring (the layout of pbn_replay_store);
 *   d_params / d_Tq the online network and its image (updated in place: Adam step, and the image
 *   of the new weights, equal to pbn_bdq_pack's bit for bit), d_target_params / d_target_Tq the
 *   target network and its image (read; the update reads the dense weights from the images); d_adam_m / d_adam_v the
 *   moments, d_adam_step float [1] Adam's step count (incremented on the device); the loss to
 *   d_loss float [1]; when d_grad is not null, the clamped gradient there.  Same arithmetic as
 *   pbn_rl_amd/replay.py bdq_update + torch.optim.Adam in fp32, to summation order.
 */
int pbn_bdq_layout(int32_t n_nodes, int32_t n_branches, int64_t* offsets);
int pbn_bdq_learn_workspace(int32_t n_nodes, int32_t n_branches, int64_t batch, int64_t* bytes);
int pbn_bdq_image_floats(const pbn_net* net, int32_t n_branches, int64_t* floats);
int pbn_bdq_pack(const pbn_net* net, int32_t n_branches, const float* d_params, float* d_Tq, void* stream);
/*
 * The learning frame's counters, advanced by the fused update's last launch (ABI 9): when
 * pbn_bdq_learn's `advance` is not null, learn_apply runs one more block that does what
 * pbn_replay_advance does for the frame just stored (position and fill level after n_store rows,
 * the env step index, epsilon's decay) and then draws the NEXT frame's n_idx rows into d_idx, over
 * the fill level that frame's store will leave (min(size + n_store, capacity)), with *d_counter,
 * which then advances.  A captured BDQ frame (pbn_rl_amd/replay.py BDQLearner) so needs no
 * launch of its own for the counters; its first rows are drawn before the first replay.  The
 * update itself reads d_idx before this block writes it (an earlier launch of the same call).
 */
typedef struct pbn_frame_advance {
  int64_t n_store, capacity;
  int64_t* d_pos;
  int64_t* d_size;
  int64_t* d_step;      /* nullable */
  double* d_eps64;      /* nullable */
  float* d_eps32;       /* nullable */
  double eps_final, eps_step;
  int64_t n_idx;
  uint64_t seed;
  int64_t* d_counter;
  int64_t* d_idx;
} pbn_frame_advance;

int pbn_bdq_learn(const pbn_net* net, int64_t batch, const int64_t* d_idx, int64_t capacity, const uint32_t* d_state,
                  const uint32_t* d_next_state, const uint8_t* d_target, const int32_t* d_action, int32_t n_branches,
                  const float* d_reward, const uint8_t* d_done, float* d_params, float* d_Tq,
                  const float* d_target_params, const float* d_target_Tq, float* d_adam_m, float* d_adam_v,
                  float* d_adam_step, float lr, float beta1, float beta2, float eps, float gamma, float grad_clamp,
                  float slope, void* d_workspace, int64_t workspace_bytes, float* d_loss, float* d_grad,
                  const pbn_frame_advance* advance, void* stream);

/*
 * pbn_copy_async (ABI 7): d_dst[0 .. bytes) <- d_src[0 .. bytes), device to device on `stream`:
 * one kernel of 16-byte non-temporal loads and stores (the world-1 hand-off of a rollout's
 * transition records, pbn_rl_amd/distributed.py; hipMemcpyAsync's blit ran 22 MB at 3.9 TB/s,
 * profiles/r05_a_handoff_summary.json).  Both pointers and `bytes` 16-byte aligned; the ranges
 * must not overlap.
 */
int pbn_copy_async(void* d_dst, const void* d_src, int64_t bytes, void* stream);

/*
 * pbn_host_buffer (ABI 9): `bytes` of pinned host memory, coherent and mapped into the current
 * device's address space (hipHostMalloc, mapped | coherent): *h_ptr is its host address, *d_ptr
 * the address kernels use; pbn_host_buffer_free releases it.  The scalar gym facade (PBNEnv,
 * one env per step, config 1) keeps its 32-env group there, so that a step is one
 * pbn_step launch on those pointers and one pbn_stream_sync, with no copies
 * (gym_PBN's env.step(), bdq_model/__init__.py:177).
 */
int pbn_host_buffer(int64_t bytes, void** h_ptr, void** d_ptr);
int pbn_host_buffer_free(void* h_ptr);
/* pbn_stream_sync (ABI 9): waits until the work issued on `stream` has completed. */
int pbn_stream_sync(void* stream);

const char* pbn_last_error(void);
int pbn_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PBN_ENV_H */
