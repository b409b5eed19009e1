/*
 * ggnn.h -- C ABI of the MI355X-native GGNN propagation engine (libggnn.so).
 *
 * Drop-in boundary for the reference's hot path
 *   DenseGGNNChemModel.compute_final_node_representations
 *   (crismolav/ggnn, chem_tensorflow_dense.py:312-340, called from
 *    chem_tensorflow.py:319-322)
 * together with its TF-autodiff backward (chem_tensorflow.py:496).
 *
 * The reference has no FFI: the path is a Python template method that builds
 * TensorFlow ops.  Each entry point below replaces one piece of that method:
 *
 *   ggnn_pack_weights   <- the path's variables, chem_tensorflow_dense.py:202-212
 *                          (edge_weights [C,h,h], edge_biases [C,1,h]) and the
 *                          GRUCell kernels/biases built at :237-241
 *   ggnn_set_adjacency  <- the adjacency placeholder + transpose, :192-195
 *                          (feed [b, C, v, v], row = receiving node, :65-83)
 *   ggnn_forward        <- the T-step loop, :312-340 = compute_timestep_fast
 *                          (:391-437) + GRUCell (:333), returns [b, v, h]
 *   ggnn_backward       <- TF autodiff of the same loop (chem_tensorflow.py:496):
 *                          dL/dh0 and the weight gradients (before clip/Adam)
 *   ggnn_dims.edge_keep / state_keep / seed
 *                       <- tf.nn.dropout of the edge weights (:397-403) and the
 *                          GRUCell DropoutWrapper (:239-240), fed at :860-861
 *
 * Conventions
 *  - Every tensor argument is a raw device pointer (hipMalloc'd or any HIP
 *    allocator, e.g. PyTorch-ROCm tensors used only as memory holders).
 *  - Host-visible layouts are the reference's: row-major fp32,
 *      adjacency [b][C][v][v] (0/1 values, row = receiver, col = sender),
 *      h0 / hT / dhT / dh0 [b][v][h],
 *      edge_weights [C][h][h] (in x out), edge_biases [C][h],
 *      gates_kernel [2h][2h] (rows [x ; h], cols [r | u]), gates_bias [2h],
 *      candidate_kernel [2h][h] (rows [x ; r*h]), candidate_bias [h].
 *  - The caller owns all memory.  The library never allocates: it works
 *    inside a caller-provided workspace sized by ggnn_workspace_bytes and a
 *    weight pack sized by ggnn_weight_pack_bytes.
 *  - All calls are asynchronous and stream-ordered on `stream`; they are safe
 *    to capture into a hipGraph (no sync, no malloc inside).
 *  - Return value: 0 on success, negative GGNN_E* on error; a description of
 *    the last error of the calling thread is in ggnn_last_error().
 *    No exception or abort crosses the ABI.
 */
#ifndef GGNN_H
#define GGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* ggnn_stream_t; /* hipStream_t (0 = default stream) */

enum {
  GGNN_OK = 0,
  GGNN_EINVAL = -1,    /* invalid dims / null pointer */
  GGNN_EUNSUP = -2,    /* dims outside the compiled kernel set */
  GGNN_ELAUNCH = -3,   /* HIP launch / runtime error */
  GGNN_EALIGN = -4     /* pointer alignment */
};

/* flags */
#define GGNN_USE_EDGE_BIAS 1 /* params['use_edge_bias'], chem_tensorflow_dense.py:158 */
/* Precision policy (fp32 accumulation in every mode).
 *   default (0)       bf16 MFMA operands, bf16 activations between kernels
 *   GGNN_FP16         f16 MFMA operands (3 more mantissa bits, same rate)
 *   GGNN_FP32_PARITY  every non-exact operand carried as an f16 hi/lo limb
 *                     pair (3 MFMAs per product, ~22-bit operand mantissa),
 *                     fp32 activations: matches the reference's fp32
 *                     arithmetic to <= 1e-3 (tests/test_gpu_parity.py).  The
 *                     backward's dz W^T / dM W_c^T products run their limb
 *                     corrections on the block-scaled fp8 MFMA (e5m2 x e4m3;
 *                     DESIGN.md §8.5); the forward keeps three f16 MFMAs */
#define GGNN_FP32_PARITY 2
#define GGNN_FP16 4
/* Empty-channel skipping.  The staged adjacency carries a
 * per-graph list of the channels with at least one edge; the message
 * transform and aggregation (forward and backward) run only over those, since
 * an empty A[g,c] contributes exactly zero (the real btb adjacency has
 * C = 2E = 92 channels, about 60 % of them empty per graph).  Results are
 * bit-identical to the dense loop.  GGNN_DENSE_CHANNELS turns the skipping
 * off (A/B measurement and the bit-identity test). */
#define GGNN_DENSE_CHANNELS 8
/* The general path (k_gemm.h + k_generic.h): any hidden size and vertex count.
 * Taken automatically when hidden is not 128 / 256 or v > 128 (e.g. the
 * reference's default hidden_size 400, chem_tensorflow.py:95, and its
 * 198-node buckets, chem_tensorflow_dense.py:584-585); GGNN_GENERIC forces it
 * for every shape (parity tests, A/B). */
#define GGNN_GENERIC 16
/* Run the forward of hidden 256, v <= 128 batches as per-timestep k_prop_fwd +
 * k_gru_fwd launches instead of the one-launch fused forward (A/B and tests). */
#define GGNN_UNFUSED_FWD 32

/* Sparse message passing on the general path ("pair mode", k_pairs.h): the
 * message transform runs over the (node, channel) pairs with an incoming edge
 * (X = sum_c (A_c h) W_c + deg beta_c, re-associated) instead of over every
 * row of every non-empty (graph, channel) tile -- the reference's dependency
 * trees have ~4 such pairs per node against ~26 non-empty channels per graph
 * (C = 92).  Same results as the dense loop up to fp32 summation order.
 * Implies GGNN_GENERIC; needs hidden % 4 == 0 and a batch staged by
 * ggnn_set_adjacency_edges with num_edges <= b * v (every edge adds at most
 * 4 pairs, so the pair buffers hold 4 * b * v rows plus channel padding);
 * ggnn_set_adjacency rejects it. */
#define GGNN_SPARSE_PAIRS 64
/* Dropout seeds live in device memory: dims.seed (and the `seed` argument of
 * ggnn_embed_* / ggnn_heads_*) holds the ADDRESS of a device uint64 that the
 * kernels read when they run, instead of the seed itself.  A step captured in
 * a hipGraph then replays with whatever seed the caller wrote there (by a
 * captured copy) -- no re-capture per training step.  Same masks as passing
 * that value directly. */
#define GGNN_SEED_DEVICE 128

typedef struct ggnn_dims {
  int32_t b;     /* graphs in the batch      (placeholders['num_graphs'])   */
  int32_t v;     /* vertices per graph       (placeholders['num_vertices']) */
  int32_t h;     /* hidden size              (params['hidden_size'])        */
  int32_t C;     /* adjacency channels = 2 * num_edge_types                 */
  int32_t T;     /* timesteps (params['num_timesteps'] or fixed_ts)         */
  int32_t flags; /* GGNN_USE_EDGE_BIAS | GGNN_FP32_PARITY or GGNN_FP16      */
  /* Dropout (applied whenever keep < 1, as the reference applies it whenever
   * a keep probability < 1 is fed; it feeds 1.0 at evaluation, :938-940):
   *   edge_keep  = placeholders['edge_weight_dropout_keep_prob']: every
   *                timestep multiplies W by a fresh mask / keep (:397-403);
   *   state_keep = placeholders['graph_state_keep_prob']: DropoutWrapper
   *                state dropout of every new GRU state (:239-240).
   * Both must lie in (0, 1].  Masks are Philox4x32-10 keyed by `seed`
   * (DESIGN.md "Dropout"), so pack, forward and backward of one step must
   * see the same seed; draw a new seed per training step. */
  float edge_keep;
  float state_keep;
  uint64_t seed;
} ggnn_dims;

int ggnn_version(void);
const char* ggnn_last_error(void);

/* Validate dims: b, v, C, T >= 1, 1 <= h <= 4096, C <= 4096.  hidden 128 / 256
 * with v <= 128 run the specialised kernels, every other shape the general
 * path.  Returns 0 or GGNN_EUNSUP / GGNN_EINVAL. */
int ggnn_check_dims(const ggnn_dims* d);

/* Bytes of the per-batch workspace (activations saved for backward when
 * training != 0), of one staged adjacency batch and of one weight pack.
 * The workspace size depends on b, v, h, C, T, flags, training and on whether
 * edge dropout is on (edge_keep < 1), not on state_keep or the seed: one
 * workspace serves every state-dropout setting of its shape. */
int ggnn_workspace_bytes(const ggnn_dims* d, int training, size_t* bytes);
int ggnn_adjacency_bytes(const ggnn_dims* d, size_t* bytes);
int ggnn_weight_pack_bytes(const ggnn_dims* d, size_t* bytes);

/* Convert fp32 master weights into the engine's MFMA fragment layouts, in the
 * precision policy of d->flags: bf16 (flag 0), f16 (GGNN_FP16) or an f16
 * hi/lo limb pair per element (GGNN_FP32_PARITY; the backward's transposed
 * packs carry e4m3 correction fragments in place of the lo limbs, clamped to
 * +-448 after their power-of-two scaling); plus the fp32 bias copies
 * and the general path's fp32 weight copies (one per timestep under edge
 * dropout, masked).  edge_biases may be NULL when !(flags & GGNN_USE_EDGE_BIAS). */
int ggnn_pack_weights(const ggnn_dims* d, void* pack,
                      const float* edge_weights, const float* edge_biases,
                      const float* gates_kernel, const float* gates_bias,
                      const float* candidate_kernel, const float* candidate_bias,
                      ggnn_stream_t stream);

/* The same pack for the batch staged in `adj` (d: that batch's dims).  On the
 * general path under edge dropout it writes the per-timestep masked copies of
 * W_c only for the channels with an edge somewhere in the batch (the others
 * are never read by that batch's forward / backward: tf.nn.dropout of
 * edge_weights, chem_tensorflow_dense.py:397-403, touches only weights the
 * batch uses).  Everything else, and other paths, as ggnn_pack_weights.  The
 * pack then serves THAT staged batch only. */
int ggnn_pack_weights_batch(const ggnn_dims* d, void* pack, const void* adj,
                            const float* edge_weights, const float* edge_biases,
                            const float* gates_kernel, const float* gates_bias,
                            const float* candidate_kernel, const float* candidate_bias,
                            ggnn_stream_t stream);

/* Test / tuning hook: D[M][N] = A[M][K] B[K][N], row-major fp32 device
 * buffers, through the general path's MFMA product kernel (k_gemm) in the
 * precision policy of d->flags (other fields of d: any valid dims). */
int ggnn_dbg_gemm(const ggnn_dims* d, int M, int N, int K, const float* A, const float* B, float* D,
                  ggnn_stream_t stream);

/* The same with every operand layout the general path uses:
 *   a_layout 0: A fp32 [M][K]; 1: A fp32 [K][M]; 2: A 16-bit limbs [M][K]
 *               (exact values: 0/1 adjacency; f16 in the fp16 / fp32 modes)
 *   b_layout 0: B fp32 [K][N]; 1: B fp32 [N][K]
 *   kernel   0: automatic; 1: k_gemm; 2: k_gemm_ring without the K split
 *               over waves; 3 / 4 / 5: k_gemm_ks (the K split) with 1 / 2 / 4
 *               column blocks of 32 (fp32 k-contiguous A).  2-5 return
 *               GGNN_EINVAL if the operands do not meet the ring's alignment
 *               rules */
int ggnn_dbg_gemm_ex(const ggnn_dims* d, int M, int N, int K, const void* A, int a_layout, const float* B,
                     int b_layout, float* D, int kernel, ggnn_stream_t stream);

/* Stage one batch's adjacency [b][C][v][v] fp32 (0/1) into `adj` (sized by
 * ggnn_adjacency_bytes): 16-bit (exact for 0/1; bf16, or f16 under GGNN_FP16 /
 * GGNN_FP32_PARITY), its transpose, per-node in-degrees and the per-graph list
 * of non-empty channels.  T of d is ignored. */
int ggnn_set_adjacency(const ggnn_dims* d, void* adj, const float* adjacency,
                       ggnn_stream_t stream);

/* Stage one batch's adjacency from edge lists instead of the dense feed (the
 * compact producer of SURVEY §8f): the same staged bytes as
 * ggnn_set_adjacency(graph_to_adj_mat_bd(...)) (chem_tensorflow_dense.py:65-83,
 * built per graph at :539) without the [b][2E][v][v] host array or its copy.
 *   edges         device int32 [num_edges][3] = (src, label, dest) rows of the
 *                 reference's 'graph' lists, graphs concatenated;
 *   graph_offsets device int32 [b + 1]: graph g owns rows [off[g], off[g+1]);
 *   num_edge_types E with d->C == 2E.
 * Labels outside 1..E or nodes outside 0..v-1 are skipped (validate on the
 * host: the reference raises IndexError for them). */
int ggnn_set_adjacency_edges(const ggnn_dims* d, void* adj, const int32_t* edges,
                             const int32_t* graph_offsets, int64_t num_edges,
                             int num_edge_types, ggnn_stream_t stream);

/* T-step forward.  h0, hT: [b][v][h] fp32.  training != 0 keeps what the
 * backward needs inside ws (ws must have been sized with training != 0). */
int ggnn_forward(const ggnn_dims* d, const void* pack, const void* adj, void* ws,
                 int training, const float* h0, float* hT, ggnn_stream_t stream);

/* Backward of the last training forward on ws (same d, pack, adj).
 * dhT, dh0: [b][v][h] fp32.  Gradient outputs are OVERWRITTEN (not
 * accumulated), fp32, reference layouts; d_edge_biases may be NULL when
 * !(flags & GGNN_USE_EDGE_BIAS). */
int ggnn_backward(const ggnn_dims* d, const void* pack, const void* adj, void* ws,
                  const float* dhT, float* dh0,
                  float* d_edge_weights, float* d_edge_biases,
                  float* d_gates_kernel, float* d_gates_bias,
                  float* d_candidate_kernel, float* d_candidate_bias,
                  ggnn_stream_t stream);

/* The reference's optimizer step for the path's variables
 * (chem_tensorflow.py:494-503): every gradient scaled by grad_scale (1/N for
 * an N-rank data-parallel mean), clipped per tensor with tf.clip_by_norm
 * (g * clip_norm / max(||g||_2, clip_norm), params['clamp_gradient_norm']),
 * then one tf.compat.v1.train.AdamOptimizer update (learning_rate,
 * beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8 in the reference):
 *   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
 *   p -= lr sqrt(1-b2^step)/(1-b1^step) m / (sqrt(v) + eps),  step >= 1.
 * scratch: device float[count * GGNN_ADAM_SCRATCH_PER_TENSOR].  Two
 * HBM-bound launches (per-tensor norms, then the update). */
#define GGNN_ADAM_SCRATCH_PER_TENSOR 256
typedef struct ggnn_adam_tensor {
  float* param;
  const float* grad;
  float* m;  /* first-moment slot, zero-initialised by the caller */
  float* v;  /* second-moment slot, zero-initialised by the caller */
  int64_t n;
  /* NULL, or a device float holding the squared norm clip_by_norm must use
   * instead of ||grad||^2 (before grad_scale): an embedding's gradient is an
   * IndexedSlices in the reference, whose norm runs over the per-lookup rows
   * (ggnn_embed_backward's lookup_sqnorm) */
  const float* sqnorm;
} ggnn_adam_tensor;
#define GGNN_ADAM_MAX_TENSORS 16
int ggnn_adam_step(const ggnn_adam_tensor* tensors, int count, float learning_rate,
                   float beta1, float beta2, float epsilon, float clip_norm,
                   int64_t step, float grad_scale, float* scratch, ggnn_stream_t stream);
/* The same with the step count read from device memory (a device int64,
 * >= 1) and the bias-corrected step size derived from it in-kernel: a step
 * captured in a hipGraph replays with whatever count the caller wrote there. */
int ggnn_adam_step_dev(const ggnn_adam_tensor* tensors, int count, float learning_rate,
                       float beta1, float beta2, float epsilon, float clip_norm,
                       const int64_t* step, float grad_scale, float* scratch,
                       ggnn_stream_t stream);

/* Materialise a dropout keep-mask (1 = kept, 0 = dropped) exactly as the
 * kernels apply it, for verification: kind 0 = edge-weight mask of timestep t
 * ([C][h][h] bytes), kind 1 = state mask of timestep t ([b][v][h] bytes). */
int ggnn_dropout_mask(const ggnn_dims* d, int kind, int t, uint8_t* mask, ggnn_stream_t stream);

/* ---- The callers either side of the path (btb task) ----
 *
 * Embedding front-end: get_initial_node_representation,
 * chem_tensorflow_dense.py:264-306.  Segment s copies row
 * word_inputs[g][i][column_s] of table_s into columns [o_s, o_s + width_s) of
 * h0[g][i] (o_s = sum of the earlier widths), times an embedding-dropout mask /
 * keep (tf.nn.dropout, keep = placeholders['emb_dropout_keep_prob']); columns
 * past the last segment are zero (the tf.pad to hidden_size, :303-305).  The
 * widths must sum to <= d->h (the reference's tf.pad fails otherwise).  Uses
 * d->b, d->v, d->h.  Rows outside [0, rows) give zero vectors (validate on the
 * host: tf.nn.embedding_lookup raises for them on the CPU). */
typedef struct ggnn_embed_segment {
  const float* table; /* [rows][width] fp32 */
  float* d_table;     /* its gradient (ggnn_embed_backward; overwritten) */
  int64_t rows;
  int32_t width;
  int32_t column;     /* column of word_inputs indexing this table */
} ggnn_embed_segment;
#define GGNN_EMBED_MAX_SEGMENTS 8
int ggnn_embed_forward(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg,
                       const int32_t* word_inputs, int ncols, float keep, uint64_t seed,
                       float* h0, ggnn_stream_t stream);
/* Gradients of the tables from dL/dh0 (+ dh0_add when not NULL: the two uses
 * of h0, the propagation input and the heads' concat), same keep and seed as
 * the forward.  lookup_sqnorm: device float[nseg] (overwritten), per TABLE the
 * sum of squares of its per-lookup gradient rows, i.e. the squared norm
 * tf.clip_by_norm takes of the reference's IndexedSlices gradient
 * (chem_tensorflow.py:498-500).  Segments sharing a d_table (btb: the loc
 * table, looked up by word_inputs columns 0 and 3) have ONE gradient whose
 * rows are both lookups' rows: their sum goes to the slot of the first such
 * segment, the later segments' slots are 0. */
int ggnn_embed_backward(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg,
                        const int32_t* word_inputs, int ncols, float keep, uint64_t seed,
                        const float* dh0, const float* dh0_add, float* lookup_sqnorm,
                        ggnn_stream_t stream);
/* The same, bit-reproducible (round 5): the lookups accumulate into a 64-bit
 * fixed-point copy of each table (2^-40 resolution, |element| < 2^23), whose
 * integer sums do not depend on the order the additions land in, and the
 * squared norms are summed in a fixed order.  ws: a device buffer of
 * ggnn_embed_workspace_bytes (which depends on the tables only, not on the
 * batch), ZERO-FILLED by the caller before its first use; every call leaves it
 * zero-filled again.  Segments sharing a d_table (which must then have one
 * shape) accumulate together, as in ggnn_embed_backward.  (ggnn_embed_backward
 * above adds fp32 atomics: its result can differ in the last bits from run to
 * run.) */
int ggnn_embed_workspace_bytes(const ggnn_embed_segment* segs, int nseg, size_t* bytes);
int ggnn_embed_backward_ws(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg,
                           const int32_t* word_inputs, int ncols, float keep, uint64_t seed,
                           const float* dh0, const float* dh0_add, float* lookup_sqnorm, void* ws,
                           ggnn_stream_t stream);
/* (ggnn_embed_backward_ws: a segment whose d_table is NULL gets no gradient
 * and a zero squared-norm slot.)
 * Segment `seg`'s gradient as the reference's IndexedSlices (values, indices;
 * chem_tensorflow.py:496-500): rows [cap][width] = the per-lookup gradient
 * rows (embedding dropout applied, keep / seed as the forward), ids [cap] =
 * the looked-up table rows (-1 out of range); rows b*v .. cap-1 are zero with
 * id -1.  The data-parallel step all-gathers these and accumulates the union
 * of every rank's lookups with ggnn_embed_backward_ws (keep 1, one segment,
 * v = 1) instead of all-reducing the dense table. */
int ggnn_embed_lookup_rows(const ggnn_dims* d, const ggnn_embed_segment* segs, int nseg, int seg,
                           const int32_t* word_inputs, int ncols, float keep, uint64_t seed,
                           const float* dh0, const float* dh0_add, float* rows, int32_t* ids,
                           int64_t cap, ggnn_stream_t stream);

/* Output heads: gated_regression for --pr btb, chem_tensorflow_dense.py:439-516
 * with MLP(2h, o, [], out_layer_dropout_keep_prob) (utils.py:40-84), and the
 * btb loss, chem_tensorflow.py:349-403:
 *   z = [h_T | h0] @ (W * mask / keep) + b      (rows = b*v nodes)
 *   probs = softmax(z) over o                    (computed_values [b, v*o])
 *   loss  = sum_rows -sum_o labels * log(probs) / target_num
 * target_num = sum(target_mask[task]) + SMALL_NUMBER (the caller's host
 * value; the _dev variants below read it from device memory).  One mask per
 * head per step (keep, seed; GGNN_SEED_DEVICE in d->flags: seed is the
 * address of a device uint64). */
typedef struct ggnn_output_head {
  const float* weight; /* MLP_W_layer0 [2h][o] */
  const float* bias;   /* MLP_b_layer0 [o] */
  int32_t o;           /* output width, 1..1024 */
  const float* labels; /* [b][v][o] targets, or NULL (no loss) */
  float* probs;        /* [b][v][o] out */
  float* d_weight;     /* [2h][o] (backward; overwritten) */
  float* d_bias;       /* [o]     (backward; overwritten) */
} ggnn_output_head;
#define GGNN_MAX_HEADS 4
int ggnn_heads_workspace_bytes(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, size_t* bytes);
/* loss: device float[nheads], overwritten (per head; the reference's loss is
 * their sum).  ws is kept for ggnn_heads_backward. */
int ggnn_heads_forward(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                       const float* h0, float keep, uint64_t seed, float target_num, float* loss,
                       void* ws, ggnn_stream_t stream);
/* d_loss: device float (dL/dloss, e.g. 1) or NULL for 1.  dhT, dh0: [b][v][h],
 * overwritten with the heads' contributions. */
int ggnn_heads_backward(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                        const float* h0, float target_num, const float* d_loss, void* ws, float* dhT,
                        float* dh0, ggnn_stream_t stream);
/* The same two with target_num read from device memory (a device float > 0),
 * for hipGraph capture of a training step: identical results to passing that
 * value (the normaliser 1 / target_num and the power-of-two scale of dZ are
 * derived from it in the kernels). */
int ggnn_heads_forward_dev(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                           const float* h0, float keep, uint64_t seed, const float* target_num, float* loss,
                           void* ws, ggnn_stream_t stream);
int ggnn_heads_backward_dev(const ggnn_dims* d, const ggnn_output_head* heads, int nheads, const float* hT,
                            const float* h0, const float* target_num, const float* d_loss, void* ws,
                            float* dhT, float* dh0, ggnn_stream_t stream);

/* Optional per-kernel timing (HIP events around every launch of the library
 * on the launch's stream), used by bench.py for the roofline.  Not for use
 * under graph capture.  total_ms / launches: arrays of GGNN_NUM_KERNEL_KINDS. */
#define GGNN_NUM_KERNEL_KINDS 11
const char* ggnn_kernel_kind_name(int kind);
int ggnn_profile_begin(int max_launches);
int ggnn_profile_end(double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif
#endif /* GGNN_H */
