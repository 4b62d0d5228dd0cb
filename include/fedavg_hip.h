/*
 * fedavg_hip.h — C ABI of the MI355X-native FedAvg aggregation path.
 *
 * This is the drop-in boundary for the server-side weighted FedAvg reduction of
 * cyyever/distributed_learning_simulation_lib. Every entry point below replaces one
 * piece of the reference's Python hot path (paths relative to the reference root):
 *
 *   fedavg_accumulate    <- FedAVGAlgorithm.process_worker_data / _accumulate_parameter
 *                           simulation_lib/algorithm/fed_avg_algorithm.py:20-64
 *   fedavg_aggregate     <- FedAVGAlgorithm._aggregate_parameter / _apply_total_weight
 *                           simulation_lib/algorithm/fed_avg_algorithm.py:71-99
 *   fedavg_weighted_avg  <- AggregationAlgorithm.weighted_avg (ratio path, accumulate=False)
 *                           simulation_lib/algorithm/aggregation_algorithm.py:51-76
 *   fedavg_partial       <- the per-shard half of _accumulate_parameter when clients are
 *                           sharded across GPUs (fp64 partial sum, no division)
 *   fedavg_*_delta       <- DeltaParameterMessage.restore fused into the fold (message.py:40-61,
 *                           aggregation_server.py:121-125)
 *   fedavg_check         <- the NaN assertions fed_avg_algorithm.py:35,93,97
 *   fedavg_find_nan_clients <- which client tripped fed_avg_algorithm.py:35
 *
 * Conventions
 *  - Plain C types only. Device pointers are `const void*` / `void*`; a stream is a
 *    `hipStream_t` passed as `void*` (NULL = the legacy default stream).
 *  - A "layout" is the ordered list of named tensors of one model (the keys of
 *    ParameterMessage.parameter, message.py:24-31). Segment t has seg_numel[t] elements.
 *  - A client table is row-major [num_clients][num_segments] of device pointers; a NULL
 *    entry means "this client did not send this tensor" (it is skipped, exactly like a
 *    missing key in the reference's per-name dictionaries, fed_avg_algorithm.py:56-62).
 *  - Weights are fp64, [num_clients][num_segments] (the value _get_weight returns for
 *    that (client, tensor), fed_avg_algorithm.py:66-69).
 *  - Accumulation is fp64 in arrival order: acc = x0*w0, then acc = acc + xk*wk, with the
 *    product and the sum each rounded (no FMA), exactly the reference's
 *    `tmp = x.to(f64) * w; acc += tmp`. Results are bit-identical to the reference for the
 *    single-GPU kernels.
 *  - Every call is asynchronous on `stream`. Arithmetic faults (NaN) are latched in a
 *    device flag and reported by fedavg_check(), which synchronises the stream.
 *  - Return value: FEDAVG_OK (0) or a negative/positive status below; the text of the
 *    last error of the calling thread is returned by fedavg_last_error().
 *  - The library never frees caller memory. Client buffers must stay valid until the
 *    call's stream work completes. One host thread per context.
 */
#ifndef FEDAVG_HIP_H
#define FEDAVG_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FEDAVG_ABI_VERSION 1

/* element types */
enum fedavg_dtype {
  FEDAVG_F32 = 0,
  FEDAVG_F16 = 1,
  FEDAVG_BF16 = 2,
  FEDAVG_F64 = 3,
  /* Quantised client records (server-side dequantisation fused into the fold,
   * StochasticQuantServerEndpoint.get, simulation_lib/topology/quantized_endpoint.py:69-77 and
   * :102-111). A client "tensor" pointer then points at one QSGD record of the tensor
   * (16-byte aligned, fedavg_qsgd_record_bytes(numel) bytes):
   *   [0, 8)   norm, fp64 (for FEDAVG_QSGD_F32 an fp32 value held exactly)
   *   [8, 12)  quantisation level s, int32 in [1, 255] (the reference uses 255)
   *   [16, 16 + numel)             slot per element, uint8 in [0, s]
   *   [fedavg_qsgd_sign_offset(numel), + ceil(numel / 8))  sign bits in numpy.packbits order
   *            (element i: byte i / 8, bit 7 - i % 8; 1 = non-negative)
   * The dequantised element is x = ((norm * sign) * slot) / s computed in fp32 (QSGD_F32) or
   * fp64 (QSGD_F64) — the codec's dtype — and is then folded exactly like a dense input
   * (tmp = x.to(f64) * w; acc += tmp). Accepted by every fold entry point except the delta
   * ones; split policies do not apply. */
  FEDAVG_QSGD_F32 = 4,
  FEDAVG_QSGD_F64 = 5,
  /* NNADQ records (NNADQServerEndpoint, quantized_endpoint.py:114-142, dequantised by
   * QuantServerEndpoint.get :69-77): a deterministic per-tensor affine code, 16-byte aligned,
   * fedavg_nnadq_record_bytes(numel) bytes:
   *   [0, 8)   lo, fp64 (for FEDAVG_NNADQ_F32 an fp32 value held exactly)
   *   [8, 16)  step, fp64 (likewise)
   *   [16, 20) levels L, int32 in [1, 255] (codes are in [0, L])
   *   [32, 32 + numel)  code per element, uint8
   * The dequantised element is x = code * step + lo (two roundings) in fp32 (NNADQ_F32) or
   * fp64 (NNADQ_F64), then folded exactly like a dense input. Same entry points as QSGD. */
  FEDAVG_NNADQ_F32 = 6,
  FEDAVG_NNADQ_F64 = 7,
};

/* status codes */
enum fedavg_status {
  FEDAVG_OK = 0,
  FEDAVG_ERR_NAN_INPUT = 1,    /* a client tensor holds NaN   (fed_avg_algorithm.py:35) */
  FEDAVG_ERR_NAN_ACCUM = 2,    /* accumulator became NaN      (fed_avg_algorithm.py:93) */
  FEDAVG_ERR_NAN_RESULT = 3,   /* acc / total_weight is NaN   (fed_avg_algorithm.py:97) */
  FEDAVG_ERR_INVALID = 4,      /* bad argument / dtype / size */
  FEDAVG_ERR_HIP = 5,          /* HIP runtime error */
  FEDAVG_ERR_STATE = 6,        /* e.g. aggregate with nothing accumulated (:88 assert) */
  FEDAVG_ERR_RCCL = 7,         /* RCCL missing or a collective failed (sharded path) */
};

/* flag bits latched by the kernels (read through fedavg_check) */
#define FEDAVG_FLAG_ACC_NAN 0x1u
#define FEDAVG_FLAG_RESULT_NAN 0x2u
#define FEDAVG_FLAG_CENTRAL_NAN 0x4u /* personalized path: the centralized average */

typedef struct fedavg_ctx fedavg_ctx;

int32_t fedavg_abi_version(void);

/* Compile-time variants the library was built with: 0 for the product build. Non-zero bits
 * mark timing-only ablation builds whose results are WRONG by design (the kernel A/B studies of
 * rounds 1-3; their sources are no longer shipped, so this build always reports 0):
 * FEDAVG_BUILD_ABLATE_EPILOGUE (reciprocal multiply, no NaN checks), FEDAVG_BUILD_ABLATE_QSGD.
 * Bindings refuse to load such a build unless asked to (_native.py). */
#define FEDAVG_BUILD_ABLATE_EPILOGUE 0x1
#define FEDAVG_BUILD_ABLATE_QSGD 0x2
int32_t fedavg_build_flags(void);

/* A compile-time constant of the kernels' geometry, by name, into *out (test support: the
 * property tests place their sizes around every edge the kernels have, derived from the build
 * instead of copied into the tests). Names: "tile", "tile_wide", "split_tile"; per input dtype
 * d in {f32, f16, bf16, f64}: "ae_<d>", "lanes_<d>" (elements per lane / lanes per tile of the
 * whole-layout table), "ae4096_<d>", "lanes4096_<d>" (the 4096-element table), "group_<d>"
 * (clients loaded per group), "pipe_<d>" (clients per pipeline stage, 0 = no pipeline);
 * "qsgd_tile", "qsgd_ae", "qsgd_group"; "nnadq_tile", "nnadq_ae", "nnadq_group",
 * "nnadq_header"; "pers_chunk", "pers_jb" (receivers per wave),
 * "pers_group" (receivers per launch), "pers_u", "pers_ring_stage", "pers_ring_depth".
 * FEDAVG_ERR_INVALID for an unknown name. */
int32_t fedavg_kernel_constant(const char* name, int64_t* out);

/* Byte size of one QSGD record of a numel-element tensor, and the offset of its sign bits
 * (see FEDAVG_QSGD_F32). Pure functions; -1 for numel < 0. */
int64_t fedavg_qsgd_record_bytes(int64_t numel);
int64_t fedavg_qsgd_sign_offset(int64_t numel);
/* Byte size of one NNADQ record of a numel-element tensor (see FEDAVG_NNADQ_F32); -1 for
 * numel < 0. */
int64_t fedavg_nnadq_record_bytes(int64_t numel);
const char* fedavg_last_error(void);

/*
 * Create a context for one model layout on one device.
 *  seg_numel[num_segments]: element count of each named tensor, in dict order.
 *  accumulator: optional caller-owned fp64 device buffer of fedavg_acc_numel() elements
 *               (e.g. a torch tensor, so a collective can run on it); NULL = the context
 *               allocates its own.
 * The fp64 accumulator uses a padded flat layout: segment t starts at
 * fedavg_segment_offset(ctx, t), a multiple of FEDAVG_ACC_ALIGN elements (256 bytes: every
 * tile boundary in accumulator coordinates is then divisible by 32, so the scatter exchange of
 * the multi-GPU round splits a chunk evenly over 2 / 4 / 8 ranks with 16-B aligned windows).
 * fedavg_layout_acc_numel gives the size before a context exists (for caller-owned buffers).
 */
#define FEDAVG_ACC_ALIGN 32
int64_t fedavg_layout_acc_numel(const int64_t* seg_numel, int32_t num_segments);
int32_t fedavg_ctx_create(fedavg_ctx** out, int32_t device, const int64_t* seg_numel,
                          int32_t num_segments, void* accumulator);
int32_t fedavg_ctx_destroy(fedavg_ctx* ctx);
int64_t fedavg_acc_numel(const fedavg_ctx* ctx);
int64_t fedavg_segment_offset(const fedavg_ctx* ctx, int32_t seg);
void* fedavg_accumulator(const fedavg_ctx* ctx);

/* Summation-order policy:
 *  1 = (default) the exact client-order kernel: bit-identical to the reference;
 *  0 = auto: the LDS split-client kernel when the layout is too small to fill the chip
 *      (< 512 tiles of 2048 elements) and a call carries >= 16 clients, else exact order;
 *  2 = the split-client kernel whenever a call carries >= 4 clients.
 * The split kernel reorders the fp64 sum (four wave partials combined in LDS). */
int32_t fedavg_set_split_policy(fedavg_ctx* ctx, int32_t policy);

/* Fused fold (default on): when every product x*w of a call is exact in fp64 — the weight's
 * significand fits next to the input's (fp32 x: weights with <= 29 significant bits, e.g.
 * integer dataset sizes < 2^29; fp16/bf16 x: <= 42 / 45 bits) — the kernel folds with one
 * fma(x, w, acc), which rounds exactly like the reference's acc + round(x*w). Otherwise (or
 * when disabled) the product and the sum are rounded separately. Results are identical
 * either way; this only trades VALU work. */
int32_t fedavg_set_fused_fold(fedavg_ctx* ctx, int32_t enable);

/* Forget accumulated state and the NaN flag (AggregationAlgorithm.clear_worker_data,
 * aggregation_algorithm.py:107-109). Asynchronous on stream. */
int32_t fedavg_reset(fedavg_ctx* ctx, void* stream);

/* Host-side per-segment total weight so far (fed_avg_algorithm.py:59-62). out[num_segments]. */
int32_t fedavg_total_weights(const fedavg_ctx* ctx, double* out);

/*
 * Streaming accumulate of a wave of clients into the fp64 accumulator, in table order.
 * Equivalent to calling _accumulate_parameter for every (client, tensor) of the wave in
 * arrival order (fed_avg_algorithm.py:43-64). Per-segment total weights accumulate on the
 * host in the same order.
 */
int32_t fedavg_accumulate(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                          const double* weights, int32_t num_clients, void* stream);

/*
 * Finish the round: optionally fold a last wave of clients (num_clients may be 0), then
 * out[t] = acc[t] / total_weight[t] converted to out_dtype (FEDAVG_F32 or FEDAVG_F64),
 * written through out_ptrs[num_segments] (device pointers). Resets the accumulator state
 * (fed_avg_algorithm.py:88-99). The acc and result NaN checks are fused in the kernel.
 * FEDAVG_ERR_STATE if nothing was ever accumulated for some segment (the :88 assert).
 */
int32_t fedavg_aggregate(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                         const double* weights, int32_t num_clients, void* const* out_ptrs,
                         int32_t out_dtype, void* stream);

/*
 * Delta updates (DeltaParameterMessage, message.py:34-61): every client tensor of the call is a
 * delta against the server's cached global model `base_ptrs[num_segments]` (fp64 device
 * tensors, e.g. the ModelCache copy, util/model_cache.py:27-34). The fold uses
 * x = base + delta (fp64, rounded — exactly restore()'s `old.to(float64) + v`, message.py:54),
 * fusing the restore into the reduce: the base is read once per tile instead of one restored
 * fp64 copy per client. Otherwise identical to fedavg_accumulate / fedavg_aggregate (arrival
 * order is preserved across mixed full/delta calls because the accumulator carries over).
 */
int32_t fedavg_accumulate_delta(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                                const double* weights, int32_t num_clients,
                                const void* const* base_ptrs, void* stream);
int32_t fedavg_aggregate_delta(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                               const double* weights, int32_t num_clients,
                               const void* const* base_ptrs, void* const* out_ptrs,
                               int32_t out_dtype, void* stream);

/*
 * Non-streaming ratio path (accumulate=False): out = sum_k ratio[k] * x_k in fp64, no
 * division (aggregation_algorithm.py:51-76). `ratios` is [num_clients][num_segments];
 * the caller computes ratios exactly like get_ratios (aggregation_algorithm.py:42-49).
 * Does not touch the accumulator.
 */
int32_t fedavg_weighted_avg(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                            const double* ratios, int32_t num_clients, void* const* out_ptrs,
                            int32_t out_dtype, void* stream);

/*
 * Multi-GPU shard step: acc[tiles in [tile_begin, tile_end)] = (acc_in ? acc : 0) +
 * sum_k w_k x_k, fp64, written to the accumulator (no division); acc_in = the context holds
 * accumulated data for the segment (earlier waves through fedavg_accumulate, or
 * fedavg_set_accumulated) and zero_init == 0. Used by the sharded
 * driver that reduces the per-GPU partials with RCCL and then calls fedavg_aggregate
 * with num_clients = 0 on the root. tile_end = -1 means "all tiles". zero_init != 0 starts
 * every segment at the additive identity -0.0 (so the shard's fold is exact, and a shard
 * without clients contributes identities).
 */
int32_t fedavg_partial(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                       const double* weights, int32_t num_clients, int32_t zero_init,
                       int32_t tile_begin, int32_t tile_end, void* stream);
/* Number of tiles and the accumulator element range [*acc_begin, *acc_end) of tiles
 * [tile_begin, tile_end), for chunking a collective over the partial. */
int32_t fedavg_num_tiles(const fedavg_ctx* ctx);
int32_t fedavg_tile_range(const fedavg_ctx* ctx, int32_t tile_begin, int32_t tile_end,
                          int64_t* acc_begin, int64_t* acc_end);
/* Declare that segments' accumulators hold data and add host totals (after an external
 * collective summed partials into the accumulator): total_weights[num_segments]. */
int32_t fedavg_set_accumulated(fedavg_ctx* ctx, const double* total_weights);
/* Finalize only tiles [tile_begin, tile_end) of the accumulator into out_ptrs (used to
 * pipeline finalize behind a chunked collective). Does not reset state. */
int32_t fedavg_finalize_range(fedavg_ctx* ctx, void* const* out_ptrs, int32_t out_dtype,
                              int32_t tile_begin, int32_t tile_end, void* stream);

/*
 * Prepared aggregation ("plan"): the client table, weights and outputs of a
 * fedavg_aggregate call are validated, compacted and uploaded ONCE; fedavg_plan_run then
 * launches the fused fold + divide with no host staging (persistent client slots, e.g. a
 * server that reuses its device buffers round after round). A run is exactly
 * fedavg_aggregate(ctx, <the planned arguments>) on a context with nothing accumulated.
 * The buffers named by the plan must outlive it.
 */
typedef struct fedavg_plan fedavg_plan;
int32_t fedavg_plan_create(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                           const double* weights, int32_t num_clients, void* const* out_ptrs,
                           int32_t out_dtype, fedavg_plan** out);
int32_t fedavg_plan_run(fedavg_plan* plan, void* stream);
int32_t fedavg_plan_destroy(fedavg_plan* plan);
/* Plans for the multi-GPU shard step, launched per tile range (chunked collective):
 * a partial plan is fedavg_partial(ctx, <clients>, zero_init, tb, te); a finalize plan is
 * fedavg_finalize_range with the given per-segment total weights baked in. */
int32_t fedavg_plan_create_partial(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                                   const double* weights, int32_t num_clients, int32_t zero_init,
                                   fedavg_plan** out);
int32_t fedavg_plan_create_finalize(fedavg_ctx* ctx, const double* total_weights,
                                    void* const* out_ptrs, int32_t out_dtype, fedavg_plan** out);
int32_t fedavg_plan_run_range(fedavg_plan* plan, int32_t tile_begin, int32_t tile_end, void* stream);

/*
 * Move accumulated state between contexts (a layout that grows when a tensor name first appears
 * in a later client, fed_avg_algorithm.py:55-62): per segment, valid[t] != 0 marks the
 * accumulator as holding data with total weight total_weights[t] (NULL: -0.0); valid[t] == 0
 * makes the next fold of that segment an assignment.
 */
int32_t fedavg_set_segment_state(fedavg_ctx* ctx, const double* total_weights, const int32_t* valid);
/* The reverse: per segment the host total weight so far and whether the accumulator holds data
 * (total_weights[num_segments], valid[num_segments]; either may be NULL). */
int32_t fedavg_segment_state(const fedavg_ctx* ctx, double* total_weights, int32_t* valid);

/*
 * Per-element weights (a _get_weight override returning a tensor of the parameter's shape,
 * fed_avg_algorithm.py:51-62, divided elementwise at :94-96):
 *   acc[e] = (acc_in ? acc[e] + round(x[e] * w[e]) : round(x[e] * w[e]))
 *   tot[e] = (acc_in ? tot[e] + w[e] : w[e]), rounded to fp32 after every add when
 *            total_fp32[t] (the reference keeps the total in the first weight's dtype)
 * weight_ptrs[K][T]: device fp32 / fp64 (weight_dtypes[K][T]) tensors of the segment's size, or
 * NULL = the scalar scalar_weights[k][t]; totals: fp64 device buffer in accumulator coordinates
 * (fedavg_acc_numel elements), owned by the caller. fedavg_finalize_elementwise writes
 * out = acc / tot (IEEE, fp32 / fp64), with the :93 / :97 NaN checks, and resets the state.
 */
int32_t fedavg_accumulate_elementwise(fedavg_ctx* ctx, const void* const* client_ptrs, int32_t in_dtype,
                                      const void* const* weight_ptrs, const int32_t* weight_dtypes,
                                      const double* scalar_weights, const int32_t* total_fp32, int32_t num_clients,
                                      void* totals, void* stream);
int32_t fedavg_finalize_elementwise(fedavg_ctx* ctx, const void* totals, void* const* out_ptrs, int32_t out_dtype,
                                    void* stream);

/* Pieces of the scatter exchange (fedavg_sharded_round_scatter; also usable from a host-driven
 * exchange, sharded.py). `finalize` is a finalize plan (its totals, outputs and out dtype).
 *  fedavg_plan_finalize_window: res[p] = src[p - lo] / W[seg(p)] for accumulator positions p in
 *      [lo, hi) that belong to a segment (padding is skipped); res is a buffer of the plan's out
 *      dtype in accumulator coordinates (fedavg_acc_numel elements); NaN checks as finalize.
 *  fedavg_plan_copy_out: the plan's outputs <- res (accumulator coordinates), every tile; a NaN
 *      in res raises the result flag (another rank's failed window reaches the root's check). */
int32_t fedavg_plan_finalize_window(fedavg_plan* finalize, const double* src, int64_t lo, int64_t hi, void* res,
                                    void* stream);
int32_t fedavg_plan_copy_out(fedavg_plan* finalize, const void* res, void* stream);
int32_t fedavg_plan_out_dtype(const fedavg_plan* plan); /* FEDAVG_F32 / FEDAVG_F64; -1 if none */

/*
 * Synchronise `stream` and report the NaN flag: FEDAVG_OK, FEDAVG_ERR_NAN_ACCUM or
 * FEDAVG_ERR_NAN_RESULT. *flags_out (optional) receives the raw flag bits.
 */
int32_t fedavg_check(fedavg_ctx* ctx, void* stream, uint32_t* flags_out);

/*
 * Diagnostic (error path only): for each client of the table, does any of its tensors hold
 * NaN? out_bad[num_clients] receives 0/1. Synchronous.
 */
int32_t fedavg_find_nan_clients(fedavg_ctx* ctx, const void* const* client_ptrs,
                                int32_t in_dtype, int32_t num_clients, int32_t* out_bad,
                                void* stream);

/* Kernel timing for bench.py: when enabled, every main-kernel launch is bracketed by a pair
 * of HIP events recorded on the launch stream. fedavg_prof_collect synchronises those
 * events, returns the summed kernel milliseconds and the launch count, and clears them. */
int32_t fedavg_prof_enable(fedavg_ctx* ctx, int32_t enable);
int32_t fedavg_prof_collect(fedavg_ctx* ctx, double* total_ms, int32_t* launches);

/* HBM ceiling probes (bench.py's measured copy / read roofline): mode 0 = 16-B copy of
 * `bytes` from src to dst, mode 1 = 16-B read-only stream of src (dst: >= 8 KiB scratch). */
int32_t fedavg_bw_probe(const void* src, int64_t bytes, void* dst, int32_t mode, void* stream);

/* =====================================================================================
 * PersonalizedFedAVG (simulation_lib/algorithm/personalized_aggregation_algorithm.py:9-57)
 *
 * Every receiver j keeps its own FedAvg over the other workers' updates, weighted by
 * worker_weights[j].get(i, 0) (:23-43); the centralized model is the equal-weight average of
 * the receivers' results in receiver order (:45-57 -> aggregation_algorithm.py:51-76).
 * One call replaces the whole round: N arrivals x M receivers, all client buckets resident.
 *
 *  client_ptrs[N][T]  arrival-ordered client tensors (NULL = the client did not send tensor t)
 *  client_ids[N]      worker id of each arrival
 *  weights[M][N]      receiver j's weight for arrival k (the .get(i, 0) value)
 *  receiver_ids[M]    worker id of each receiver (unique; receiver order = key order): receiver
 *                     j skips the arrivals whose id equals its own (:31-32)
 *  out_ptrs[M][T]     receiver results: acc_j / W_j (fed_avg_algorithm.py:71-99), fp32 or fp64
 *  central_ptrs[T]    optional: sum_j round(out_j * (1/M)) in receiver order, fp32 or fp64
 * Per receiver and segment the sum is the reference's arrival-order fp64 chain with separately
 * rounded products (fused to one fma only when the host proves every product exact), so every
 * output is bit-identical to the reference's float64 result (the fp32 outputs: its cast).
 * FEDAVG_ERR_STATE when a receiver folds no client for some segment (the :88 assertion). NaN
 * conditions (input NaN, inf*0, 0/0, inf-inf) latch flags reported by fedavg_pers_check.
 * ===================================================================================== */
typedef struct fedavg_pers fedavg_pers;
int32_t fedavg_pers_create(fedavg_pers** out, int32_t device, const int64_t* seg_numel, int32_t num_segments);
int32_t fedavg_pers_destroy(fedavg_pers* p);
/* fused fold when every product is provably exact (default on; results identical either way) */
int32_t fedavg_pers_set_fused_fold(fedavg_pers* p, int32_t enable);
int32_t fedavg_pers_aggregate(fedavg_pers* p, const void* const* client_ptrs, int32_t in_dtype,
                              int32_t num_clients, const int64_t* client_ids, const double* weights,
                              const int64_t* receiver_ids, int32_t num_receivers,
                              void* const* out_ptrs, int32_t out_dtype, void* const* central_ptrs,
                              int32_t central_dtype, void* stream);
/* Synchronise `stream`, report and clear the NaN flags (FEDAVG_FLAG_*): FEDAVG_OK,
 * FEDAVG_ERR_NAN_ACCUM (a receiver's accumulator: input NaN, inf*0, inf-inf) or
 * FEDAVG_ERR_NAN_RESULT (a receiver's result, e.g. 0/0, or the centralized average). */
int32_t fedavg_pers_check(fedavg_pers* p, void* stream, uint32_t* flags_out);
int32_t fedavg_pers_prof_enable(fedavg_pers* p, int32_t enable);
int32_t fedavg_pers_prof_collect(fedavg_pers* p, double* total_ms, int32_t* launches);
/* fp64 VALU ceiling probe (independent v_fma_f64 chains): measured TFLOP/s */
int32_t fedavg_fp64_probe(int64_t waves, int32_t iters, double* tflops_out, void* stream);

/* =====================================================================================
 * Host ingest (aggregation_server.py:129: updates arrive as CPU tensors). Copy one client's
 * n tensors (pageable host memory, srcs[i], nbytes[i]) into a pinned staging bucket at byte
 * offsets dst_off[i], with a persistent pool of host threads (FEDAVG_PACK_THREADS, default
 * min(OMP_NUM_THREADS or cores, 8)); the caller then moves the bucket with one DMA.
 * Synchronous. A NULL source or 0 bytes is skipped.
 * ===================================================================================== */
int32_t fedavg_host_pack(void* dst, const void* const* srcs, const int64_t* nbytes, const int64_t* dst_off,
                         int32_t n);
int32_t fedavg_host_pack_threads(void);

/* =====================================================================================
 * Multi-GPU exchange step (replaces nothing in the reference, which
 * sends every update to one server process: aggregation_server.py:111-145). One process per
 * GPU; the library owns an RCCL communicator (bound at run time from the process's RCCL,
 * librccl.so.1 — torch's when torch is loaded; FEDAVG_RCCL_LIB overrides).
 *   rank 0: fedavg_comm_unique_id(id); the caller ships the FEDAVG_COMM_ID_BYTES to every rank
 *   every rank: fedavg_comm_create(&comm, id, world, rank, device)   (collective)
 *   every round: fedavg_sharded_round(comm, ctx, partial_plan, finalize_plan_or_NULL, chunks,
 *                root, stream)
 * A round launches the partial plan in `chunks` tile ranges on `stream`; after each range its
 * fp64 partial is summed into the root's accumulator by ncclReduce on the communicator's
 * high-priority stream (overlapping the next range's kernel); `stream` then waits for the last
 * reduce and the root runs the finalize plan over every tile. Asynchronous; check with
 * fedavg_check on the root. Results: each rank's fold is exact, the cross-rank fp64 sum is
 * RCCL's order. With profiling enabled on ctx, only the first chunk's launch of
 * a round is timed (fedavg_prof_collect).
 * ===================================================================================== */
#define FEDAVG_COMM_ID_BYTES 128
typedef struct fedavg_comm fedavg_comm;
int32_t fedavg_comm_unique_id(void* id_out);
int32_t fedavg_comm_create(fedavg_comm** out, const void* id, int32_t world, int32_t rank, int32_t device);
int32_t fedavg_comm_destroy(fedavg_comm* comm);
int32_t fedavg_sharded_round(fedavg_comm* comm, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                             int32_t chunks, int32_t root, void* stream);
/*
 * The same round with a scatter exchange instead of a reduce to the root (DESIGN.md §5 cost
 * table). Every rank passes a finalize plan (non-root ranks: scratch outputs of the same
 * layout). Per chunk [A, B) of the accumulator (B - A = G*L + R):
 *   ncclReduceScatter of acc[A, A + G*L) (rank r receives the sums of window
 *   [A + r*L, A + (r+1)*L)) — plus, when R > 0, an ncclReduce of the R-element tail to the root,
 *   in one group — on the comm stream behind the chunk's partial kernel; each rank divides its
 *   window (fedavg_plan_finalize_window) and ncclGather collects the windows, in the output dtype,
 *   into the root's result buffer (accumulator coordinates). `stream` then waits for the last
 *   gather and the root copies the result into its outputs (fedavg_plan_copy_out). A NaN on any
 *   rank's window surfaces in the root's fedavg_check (as FEDAVG_ERR_NAN_RESULT).
 * Root ingress: (G-1)/G of the fp64 partial + (G-1)/G of the result, against the whole fp64
 * partial for fedavg_sharded_round; every rank egresses the same (G-1)/G of its partial.
 */
int32_t fedavg_sharded_round_scatter(fedavg_comm* comm, fedavg_ctx* ctx, fedavg_plan* partial,
                                     fedavg_plan* finalize, int32_t chunks, int32_t root, void* stream);
/*
 * Either round with caller-chosen chunks: tile_edges[0..num_edges) runs from 0 to
 * fedavg_num_tiles(ctx), strictly increasing; chunk k is tiles [tile_edges[k], tile_edges[k+1]).
 * Uneven chunks shift the exposed part of the exchange: a short last chunk shortens the tail when
 * the exchange keeps up with the fold, a short first chunk starts the exchange sooner when it
 * does not (sharded.tune_exchange times the shapes on the node). exchange: FEDAVG_EXCHANGE_*.
 * fedavg_sharded_round(..., chunks, ...) is this call with `chunks` equal ranges.
 */
#define FEDAVG_EXCHANGE_REDUCE 0
#define FEDAVG_EXCHANGE_SCATTER 1
int32_t fedavg_sharded_round_edges(fedavg_comm* comm, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                                   const int32_t* tile_edges, int32_t num_edges, int32_t exchange, int32_t root,
                                   void* stream);

/* =====================================================================================
 * Dynamic waves — the round's first wave folded while its clients still arrive.
 * Replaces, for the plugin's round (FedAVGAlgorithm.process_worker_data x N then
 * aggregate_worker_data, simulation_lib/algorithm/fed_avg_algorithm.py:20-113, driven by
 * simulation_lib/server/aggregation_server.py:111-145), the wave that could only start once every
 * arrival was staged: the kernel is launched at the first arrival with an open client count.
 *
 *   fedavg_dyn_open(ctx, in_dtype, max_clients, stream)
 *       launch the wave (zero-initialised: the accumulator must hold nothing yet) on a private
 *       stream, behind what `stream` holds so far. While it is open every other launch on the
 *       context fails with FEDAVG_ERR_STATE.
 *   fedavg_dyn_publish(ctx, client_ptrs[K][T], weights[K][T], K, stream, &published)
 *       hand rows [already published, K) of the caller's client table to the wave (rows keep
 *       their indices: the same table the caller appends to). Rows must carry every tensor, 16-B
 *       aligned, one weight per row (else FEDAVG_ERR_INVALID: close the wave and fold the rest
 *       the ordinary way). Nothing is published (published = 0) while `stream` has unfinished
 *       work — the tensors of those rows may not be written yet.
 *   fedavg_dyn_close(ctx, out_ptrs or NULL, out_dtype, join, stream, &folded, &finalized)
 *       fix the count. With out_ptrs (16-B aligned) the wave divides by the published rows'
 *       totals (arrival order) into the outputs: finalized = 1, the round is done (check with
 *       fedavg_check on `stream`). Otherwise — NULL outputs, or the wave ended itself after
 *       FEDAVG_DYN_IDLE_US (200) µs without a new row or FEDAVG_DYN_LIFE_US (2 s) in all — it
 *       stores the fp64 accumulator of rows [0, folded) (the context's state says so) and the
 *       caller folds rows [folded, K) with the ordinary calls; `stream` then continues after the
 *       wave. A finalized wave with join = 1 likewise orders `stream` after it; with join = 0
 *       it does not — the outputs are complete once the next fedavg_check on this context
 *       returns (it waits for the wave), which spares `stream` the cross-stream wait (a stream
 *       that waited on another's event can still read as busy right after its synchronize).
 *       folded counts the caller's rows from 0 (every wave of the round, see below).
 *   A wave that ended itself stays open for the caller: the next publication that hands over
 *       rows launches a fresh wave continuing from the fp64 accumulator (its rows [0, folded) are
 *       there) — the reference server's poll loop hands updates over in bursts with a sleep in
 *       between (simulation_lib/server/server.py:133-146), and each burst after the idle limit is
 *       folded while it arrives. Rows published to the ended wave after it stopped reading are
 *       handed to the new one. The close divides by the totals of every published row.
 *   fedavg_dyn_state(ctx, &active, &published)
 *   fedavg_dyn_info(ctx, info, n): the first n of {active, published, rows in the accumulator from
 *       waves that ended themselves this round, continued waves (cumulative), wave launches
 *       (cumulative)}.
 * Per element the fold is the reference's arrival-order chain (separately rounded product and
 * sum): the bits equal fedavg_aggregate's.
 * ===================================================================================== */
int32_t fedavg_dyn_open(fedavg_ctx* ctx, int32_t in_dtype, int32_t max_clients, void* stream);
int32_t fedavg_dyn_publish(fedavg_ctx* ctx, const void* const* client_ptrs, const double* weights, int32_t num_clients,
                           void* stream, int32_t* published_out);
int32_t fedavg_dyn_close(fedavg_ctx* ctx, void* const* out_ptrs, int32_t out_dtype, int32_t join, void* stream,
                         int32_t* folded_out, int32_t* finalized_out);
int32_t fedavg_dyn_state(const fedavg_ctx* ctx, int32_t* active, int32_t* published);
int32_t fedavg_dyn_info(const fedavg_ctx* ctx, int32_t* info, int32_t n);
/* GPU-clock timing of the context's last wave when it ran with fedavg_prof_enable on (each tile
 * workgroup then stores its finishing time; this call waits for the wave and reads them): the first
 * n of {µs from the mirror handing the tiles their last rows to the wave's last workgroup finishing
 * (the fold after the last publication, result stores included), µs from the mirror seeing the
 * close to that end, µs from the last rows to the close} — -1 where not recorded. */
int32_t fedavg_dyn_timing(const fedavg_ctx* ctx, double* out, int32_t n);
/* The wave's idle limit and lifetime in microseconds for the following launches (0 keeps the
 * current value; the defaults come from FEDAVG_DYN_IDLE_US / FEDAVG_DYN_LIFE_US, 200 us / 2 s). */
int32_t fedavg_dyn_configure(fedavg_ctx* ctx, int64_t idle_us, int64_t life_us);
/* With fedavg_prof_enable on: the summed time of the closed waves' body launches (enqueue at
 * the open to the launch's end, so the arrival phase is included) and their count; clears them. */
int32_t fedavg_dyn_prof_collect(fedavg_ctx* ctx, double* total_ms, int32_t* waves);

/* =====================================================================================
 * Single-process multi-device mode ("a communicator created by the library
 * from a device list"). The reference drives aggregation from ONE server process
 * (simulation_lib/server/server.py:122-152 -> aggregation_server.py:111-145 ->
 * FedAVGAlgorithm.process_worker_data / aggregate_worker_data, fed_avg_algorithm.py:20-113);
 * this object lets that one process shard the sum of fed_avg_algorithm.py:43-64 over G MI355X.
 *
 *   fedavg_multi_create(&m, devices, G, seg_numel, T, accumulators_or_NULL)
 *       one context per device entry (fedavg_multi_context: fold that device's shard with the
 *       single-device calls above), one library stream and one high-priority exchange stream per
 *       entry, peer access enabled between distinct devices (fedavg_multi_peer_access). Entries
 *       may repeat a device (aliased devices: tests on one GPU).
 *   fedavg_multi_round(m, partials[G], totals, outs, out_dtype, root, edges, n_edges, exchange,
 *                      streams)
 *       one round of device-resident clients: partials[g] is a zero-initialised partial plan on
 *       context g (NULL = device g holds no client). Exchanges:
 *        FEDAVG_EXCHANGE_PEER  — chunk k (tiles [edges[k], edges[k+1])) is cut into G windows,
 *          device j owns window j. Device g's partial kernel for window j != g stores its fp64
 *          partial straight into device j's receive slot over xGMI; device j then folds its own
 *          window and, in the same kernel, sums the G partials of it in device order
 *          S_0 + S_1 + ... (its own from registers; deterministic), divides by totals[t] and
 *          stores the result into the root's outputs (a peer store). Cross-device order is
 *          carried by events (no spinning kernel). Needs peer access (or aliased devices).
 *        FEDAVG_EXCHANGE_REDUCE — each chunk's partials are reduced to the root's accumulator by
 *          an in-process RCCL communicator (ncclCommInitAll, created on first use; RCCL's
 *          summation order), then the root divides.
 *       streams[g]: the caller's stream of entry g (NULL = the library's); each entry's work is
 *       ordered after what the caller enqueued there before, and streams[root] is ordered after
 *       the whole round.
 *   fedavg_multi_combine(m, totals, outs, out_dtype, root, exchange, streams)
 *       the streaming form: every context's accumulator already holds its shard's fp64 partial
 *       (folded in waves with fedavg_accumulate on context g); segments a context never folded
 *       count as the identity. FEDAVG_ERR_STATE if no context folded some segment (the :88
 *       assertion). Resets every context's accumulated state (fed_avg_algorithm.py:90,98).
 *   fedavg_multi_check(m, flags_out): synchronise every stream of the object and report the OR
 *       of every context's NaN flags like fedavg_check; fedavg_multi_reset clears them.
 *   fedavg_multi_round_check(m, flags_out): the same report after waiting for the end of the
 *       last round / combine only (one event, behind every entry's exchange work) — the per-round
 *       form of the reference's assertions (fed_avg_algorithm.py:35,93,97) for a server that
 *       enqueued nothing else on the object's streams since; fedavg_multi_check before any round.
 * Results: each device's fold is the exact arrival-order chain of its clients; PEER sums the
 * partials in device order (bit-identical to that host composition), REDUCE in RCCL's order.
 * Every call returns with the caller's current device (hipGetDevice) unchanged. Destroy the
 * plans made on the entries' contexts before (or after) fedavg_multi_destroy: a plan keeps its
 * device, not its context, for its own destroy, but must not be run once the object is gone.
 * ===================================================================================== */
#define FEDAVG_EXCHANGE_PEER 2
#define FEDAVG_MULTI_MAX_DEVICES 16
typedef struct fedavg_multi fedavg_multi;
int32_t fedavg_multi_create(fedavg_multi** out, const int32_t* devices, int32_t num_devices, const int64_t* seg_numel,
                            int32_t num_segments, void* const* accumulators);
int32_t fedavg_multi_destroy(fedavg_multi* m);
int32_t fedavg_multi_num_devices(const fedavg_multi* m);
int32_t fedavg_multi_device(const fedavg_multi* m, int32_t index);
fedavg_ctx* fedavg_multi_context(fedavg_multi* m, int32_t index);
void* fedavg_multi_stream(fedavg_multi* m, int32_t index);
/* 1 when every pair of distinct devices of the object has peer access enabled, else 0 */
int32_t fedavg_multi_peer_access(const fedavg_multi* m);
int32_t fedavg_multi_round(fedavg_multi* m, fedavg_plan* const* partials, const double* total_weights,
                           void* const* out_ptrs, int32_t out_dtype, int32_t root, const int32_t* tile_edges,
                           int32_t num_edges, int32_t exchange, void* const* streams);
int32_t fedavg_multi_combine(fedavg_multi* m, const double* total_weights, void* const* out_ptrs, int32_t out_dtype,
                             int32_t root, int32_t exchange, void* const* streams);
int32_t fedavg_multi_check(fedavg_multi* m, uint32_t* flags_out);
int32_t fedavg_multi_round_check(fedavg_multi* m, uint32_t* flags_out);
int32_t fedavg_multi_reset(fedavg_multi* m);
/* Measurement of fedavg_multi_round (bench.py's N > 1 line): while enabled, every round records
 * three timing events on entry 0's stream (device 0) — the round's start, the end of entry 0's
 * last chunk fold (its client reads; the peer stores of its other windows), and the round's end
 * behind every entry's exchange work. fedavg_multi_prof_collect waits for them and returns the
 * summed fold and tail (fold end -> round end: the exposed exchange + division that the
 * reference's single server process, simulation_lib/server/server.py:122-152, waits for after the
 * last fold) times in ms over the recorded rounds, then clears them. The markers sit between the
 * round's launches, so time profiled rounds apart from the timed ones. */
int32_t fedavg_multi_prof_enable(fedavg_multi* m, int32_t on);
int32_t fedavg_multi_prof_collect(fedavg_multi* m, double* fold_ms, double* tail_ms, int32_t* rounds);

#ifdef __cplusplus
}
#endif

#endif /* FEDAVG_HIP_H */
