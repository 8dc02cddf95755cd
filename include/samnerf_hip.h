/*
 * samnerf_hip.h -- C ABI of the MI355X (gfx950) NeRF ray-march library
 * (libsamnerf_hip.so).  Plain pointers and sizes only; no torch types.
 *
 * All pointers are DEVICE pointers unless a parameter says "host".  Every
 * function is asynchronous on `stream` (a hipStream_t; NULL = the legacy
 * default stream, which is what the reference's <<<>>> launches use,
 * gridencoder.cu:386), never synchronises the host, never allocates, and
 * returns 0 on success or a negative SAMNERF_E* code; the message is then
 * available from samnerf_last_error() (thread-local).
 *
 * Drop-in encoder entry points -- one per pybind function of the reference:
 *   gridencoder/src/gridencoder.h:12-16 (bound at gridencoder/src/bindings.cpp:6-9)
 *   shencoder/src/shencoder.h:9-10      (bound at shencoder/src/bindings.cpp:6-7)
 *   freqencoder/src/freqencoder.h:7,10  (bound at freqencoder/src/bindings.cpp:6-7)
 * Argument order and meaning follow those signatures; tensors become raw
 * float / int32 pointers (fp32 only: the reference's fp16 dispatch is dead on
 * this path because main.py:222 forces fp16 off).
 *
 * Fused entry points -- the ray-march inner loop of nerf/renderer.py:221-390
 * + nerf/network.py:221-259 (NeRFRenderer.run), which the reference runs as
 * ~350 unfused ATen ops per chunk around the encoder kernels.
 */
#ifndef SAMNERF_HIP_H
#define SAMNERF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* samnerf_stream_t; /* == hipStream_t */

enum {
    SAMNERF_OK = 0,
    SAMNERF_EINVAL = -1,   /* bad argument (shape / enum / null pointer) */
    SAMNERF_ELAUNCH = -2,  /* kernel launch failed */
    SAMNERF_EWORKSPACE = -3 /* workspace too small */
};

/* Library identity / diagnostics (host only, no GPU needed). */
const char* samnerf_version(void);
const char* samnerf_last_error(void);
/* 1 in the diagnostic build (libsamnerf_hip_diag.so: the kernels' A/B variant
 * switches read from SAMNERF_* environment variables, for the bit-identity
 * tests), 0 in the product library (one path per configuration). */
int samnerf_diag_variants(void);

/* ------------------------------------------------------------ gridencoder --
 * Replaces grid_encode_forward (gridencoder.h:12, gridencoder.cu:467-490).
 * inputs [B,D] in [0,1]; embeddings [rows,C]; offsets [L+1] int32;
 * outputs [L,B,C] (level-major, as grid.py:49 allocates it); dy_dx
 * [B, L*D*C] or NULL.  gridtype 0 hash / 1 tiled; interp 0 linear /
 * 1 smoothstep.  Levels >= max_level are not written (caller zero-fills,
 * grid.py:52).  C in {1,2,4,8,16,32}, D in {2,3,4,5}. */
int samnerf_grid_encode_forward(const float* inputs, const float* embeddings,
                                const int32_t* offsets, float* outputs,
                                uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                uint32_t max_level, float S, uint32_t H,
                                float* dy_dx, uint32_t gridtype, int align_corners,
                                uint32_t interp, samnerf_stream_t stream);

/* Replaces grid_encode_backward (gridencoder.h:13, gridencoder.cu:492-522).
 * grad [L,B,C]; grad_embeddings [rows,C] accumulated into (caller zeroes,
 * grid.py:83); dy_dx / grad_inputs both NULL or both set ([B,D], written). */
int samnerf_grid_encode_backward(const float* grad, const float* inputs,
                                 const float* embeddings, const int32_t* offsets,
                                 float* grad_embeddings, uint32_t B, uint32_t D,
                                 uint32_t C, uint32_t L, uint32_t max_level, float S,
                                 uint32_t H, const float* dy_dx, float* grad_inputs,
                                 uint32_t gridtype, int align_corners, uint32_t interp,
                                 samnerf_stream_t stream);

/* Replaces grad_total_variation (gridencoder.h:15, gridencoder.cu:662-668). */
int samnerf_grad_total_variation(const float* inputs, const float* embeddings, float* grad,
                                 const int32_t* offsets, float weight, uint32_t B,
                                 uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                 uint32_t gridtype, int align_corners,
                                 samnerf_stream_t stream);

/* Replaces grad_weight_decay (gridencoder.h:16, gridencoder.cu:705-713).
 * B = rows of the embeddings table. */
int samnerf_grad_weight_decay(const float* embeddings, float* grad, const int32_t* offsets,
                              float weight, uint32_t B, uint32_t C, uint32_t L,
                              samnerf_stream_t stream);

/* -------------------------------------------------------------- shencoder --
 * Replaces sh_encode_forward (shencoder.h:9, shencoder.cu:400-417).
 * inputs [B,D=3] unit vectors; outputs [B,C*C] (C = degree 1..8);
 * dy_dx [B,D,C*C] or NULL. */
int samnerf_sh_encode_forward(const float* inputs, float* outputs, uint32_t B, uint32_t D,
                              uint32_t C, float* dy_dx, samnerf_stream_t stream);

/* Replaces sh_encode_backward (shencoder.h:10, shencoder.cu:419-438).
 * grad_inputs [B,D] is accumulated into (caller zeroes, sphere_harmonics.py:50). */
int samnerf_sh_encode_backward(const float* grad, const float* inputs, uint32_t B, uint32_t D,
                               uint32_t C, const float* dy_dx, float* grad_inputs,
                               samnerf_stream_t stream);

/* ------------------------------------------------------------ freqencoder --
 * Replaces freq_encode_forward (freqencoder.h:7, freqencoder.cu:97-110):
 * outputs [B, C], C = D + 2*D*deg. */
int samnerf_freq_encode_forward(const float* inputs, uint32_t B, uint32_t D, uint32_t deg,
                                uint32_t C, float* outputs, samnerf_stream_t stream);

/* Replaces freq_encode_backward (freqencoder.h:10, freqencoder.cu:113-129). */
int samnerf_freq_encode_backward(const float* grad, const float* outputs, uint32_t B,
                                 uint32_t D, uint32_t deg, uint32_t C, float* grad_inputs,
                                 samnerf_stream_t stream);

/* ------------------------------------------------------ ray-march pieces --
 * Stand-alone kernels of the individual steps, used by the parity tests and
 * by hosts that keep their own loop.  Each cites the reference op sequence it
 * reproduces. */

/* get_rays, full-image branch (nerf/utils.py:145-279, N = -1):
 * pose_host = row-major 4x4 cam2world (host), intrinsics (fx, fy, cx, cy);
 * rays_o, rays_d [rows*W, 3]: the rays of pixel rows [row0, row0 + rows). */
int samnerf_get_rays(const float* pose_host, float fx, float fy, float cx, float cy,
                     uint32_t H, uint32_t W, uint32_t row0, uint32_t rows,
                     float* rays_o, float* rays_d, samnerf_stream_t stream);

/* near_far_from_aabb (nerf/renderer.py:122-139); aabb_host = 6 floats. */
int samnerf_near_far(const float* rays_o, const float* rays_d, uint32_t N,
                     const float* aabb_host, float min_near, float* nears, float* fars,
                     samnerf_stream_t stream);

/* contract (nerf/renderer.py:60-69): x, z [N,3]. */
int samnerf_contract(const float* x, float* z, uint32_t N, samnerf_stream_t stream);

/* sample_pdf (nerf/renderer.py:84-119, perturb = False): bins [N,T0+1],
 * weights [N,T0] -> out [N,T]; inds [N,T] int32 (searchsorted result, may be
 * NULL). */
int samnerf_sample_pdf(const float* bins, const float* weights, uint32_t N, uint32_t T0,
                       uint32_t T, float* out, int32_t* inds, samnerf_stream_t stream);

/* sigmas -> weights (nerf/renderer.py:310-326, background 'last_sample'):
 * real_bins [N,T+1], sigmas [N,T] -> weights [N,T]. */
int samnerf_composite_weights(const float* real_bins, const float* sigmas, uint32_t N,
                              uint32_t T, float* weights, samnerf_stream_t stream);

/* Host helper: torch.linspace(start, end, steps) in float32 exactly as torch
 * computes it on the CPU (the sample positions of renderer.py:97, :265). */
void samnerf_linspace_host(float start, float end, uint32_t steps, float* out_host);

/* ------------------------------------------------------------ fused path --
 * One hash grid of the model (GridEncoder, gridencoder/grid.py:102-146). */
typedef struct {
    const float* embeddings;      /* device [rows, level_dim] */
    const int32_t* offsets_host;  /* HOST [num_levels + 1] (grid.py:124-135) */
    uint32_t num_levels;
    uint32_t level_dim;
    float S;                      /* log2(per_level_scale), grid.py:38 */
    uint32_t base_resolution;     /* H */
} samnerf_grid;

/* NeRFNetwork(opt) weights (nerf/network.py:94-219), torch layout [out, in],
 * plus the forced options of main.py:222-226. */
typedef struct {
    samnerf_grid grid;            /* network.py:102  L16 C2  */
    samnerf_grid s_grid;          /* network.py:111  L16 C8  (with_sam) */
    samnerf_grid prop[2];         /* network.py:211, :216  L5 C2 */
    const float* grid_mlp[3];     /* [64,32] [64,64] [16,64] */
    const float* view_mlp[3];     /* [32,31] [32,32] [3,32]  */
    const float* prop_mlp[2][2];  /* [16,10] [1,16] each */
    const float* sam_w[5];        /* [256,163] [256,256] [256,419] [256,256] [256,256] */
    const float* sam_b[5];        /* [256] each */
    const float* ln_w;            /* LayerNorm(256) weight / bias */
    const float* ln_b;
    int with_sam;
    float aabb[6];                /* aabb_infer (renderer.py:163-167) */
    float grid_bound;             /* 2 under contract (renderer.py:152-153) */
    float min_near;               /* main.py:69 */
    uint32_t num_steps[3];        /* (128, 64, 32), main.py:79-80 */
    int head_mode;                /* precision of the GEMMs -- grid_mlp (per sample), the SAM
                                     head and the mask head: 0 = f16x3, each fp32 product as
                                     three fp16 MFMA products on power-of-two scaled operands
                                     with fp32 accumulate (fp32-equivalent, default); 1 = exact
                                     fp32 MFMA (v_mfma_f32_32x32x2_f32) */
    float t_thresh;               /* N1, a flagged NON-PARITY mode: 0 = off (the
                                     reference's semantics, default); t in (0, 1): a wave of 32
                                     rays stops marching the final stage once every ray's
                                     transmittance is below t -- the dropped samples' weights
                                     (their sum <= t per ray) become 0, so weights_sum, depth,
                                     colour and features change by at most t x their range */
    uint32_t view_width;          /* layout hint of the ray batch, not a weight: the rays are a
                                     row-major image this many pixels wide (0 = unknown).  When W
                                     is a multiple of 8 and N of 4 W, the kernels group rays into
                                     8 x 4 pixel tiles (compact wave footprints, better gather
                                     locality); outputs stay in ray order and are bit-identical.
                                     samnerf_sgrid_backward must see the value of the forward. */
    /* --with_mask instance heads (network.py:125-203, renderer.py:392-452), rendered by
     * samnerf_mask_forward after a samnerf_render_forward with with_mask = 1 (0: no mask
     * outputs, nothing extra computed).  mask_kind 0 = 'default': m_grid L16 C8 and
     * SkipConnMLP(143 -> 256 -> 256 -> mask_out, bias=False, leaky_relu), mask_w[0..2]
     * = [256,143] [256,256] [mask_out,256]; 1 = 'adaptive' / 'density': six bias-free
     * Linears on the grid_mlp intermediates, mask_w[0..5] = [96,32] [96,160] [96,160]
     * [96,112] [96,96] [mask_out,96]; 2 = 'adaptive' / 'rgb' (needs sum_after_mlp):
     * eight, also on the view_mlp intermediates, mask_w[0..7] = [96,32] [96,160]
     * [96,160] [96,112] [96,128] [96,128] [96,96] [mask_out,96].
     * with_mask = 2: a training render -- the adaptive heads' render also keeps
     * each ray's weighted input sums (240 floats per ray) in the workspace for
     * samnerf_mask_train_forward / _backward, which need with_mask = 2 on those
     * heads; inference renders (1) neither store nor allocate them. */
    int with_mask;
    int mask_kind;
    samnerf_grid m_grid;          /* mask_kind 0 */
    const float* mask_w[8];
    uint32_t mask_out;            /* n_inst (+ redundant_instance for 'default'), 1..32 */
    int sum_after_mlp;            /* --sum_after_mlp (renderer.py:339-342): image =
                                     sigmoid(sum_k w_k view_mlp(colour_k)); RGB / mask models only
                                     (with SAM features the reference crashes) */
    /* perturb=True (renderer.py:266-271 and sample_pdf's :100-101): the perturbed
     * sample positions as the reference computes them from torch.rand_like, ray order:
     * perturb[0] = the stage-0 bins clamp(linspace(0, 1, T0+1) + (rand - 0.5) / T0, 0, 1)
     * [N][num_steps[0]+1]; perturb[1], perturb[2] = sample_pdf's u = linspace(0.5/T,
     * 1-0.5/T, T) + (rand - 0.5) / T of stages 1 and 2, [N][T] with T = num_steps[s]+1.
     * Set per call; all NULL = perturb=False (the default), all three or none. */
    const float* perturb[3];
    /* 1: the render workspace already holds this model's packed MLP weights
     * (the f16x3 grid_mlp fragments and the SAM head's weight stream) from an
     * earlier samnerf_render_forward(_tile) on the same workspace with the same
     * weights and head_mode, so the packing launches (k_pack_grid_mlp,
     * k_head_wmax, k_pack_h16: ~25 us per call) are skipped; 0 (default):
     * pack.  The caller vouches for it (fused.py: the weights' data pointers
     * and torch version counters); the diagnostic library always packs. */
    int reuse_packed;
} samnerf_model;

/* Bytes of device workspace samnerf_render_forward needs for N rays. */
size_t samnerf_render_workspace_size(const samnerf_model* model, uint32_t N);

/* The whole ray-march inner loop for N rays (NeRFRenderer.run in eval mode:
 * perturb = False unless model->perturb is set, background 'last_sample', sum_after_mlp = False,
 * sam_use_view_direction = True): near/far, 3 proposal rounds with
 * inverse-CDF resampling, hash-grid + SH encoding, sigma / colour MLPs,
 * compositing, view MLP, and (with_sam) the s_grid feature composite plus the
 * SkipConnMLP + LayerNorm head.
 *   rays_o, rays_d [N,3]; cam_near_far [N,2] or [1,2] (n_cnf rows) or NULL;
 *   bg_color: scalar background (renderer.py:239-240, default 1);
 *   image [N,3], depth [N], weights_sum [N]; samvit [N,256] (with_sam; NULL
 *   = features not wanted: the s_grid composite and the head are skipped --
 *   renderer.py computes and drops them when return_feats == 0);
 *   feature_rows [N,164] optional: the per-ray head input
 *   cat(f_sam, f_image, image, depth) (+1 pad), kept for training.
 * Outputs are written, never accumulated.  N = 0 returns SAMNERF_OK without
 * touching any buffer (they may be NULL). */
int samnerf_render_forward(const samnerf_model* model, const float* rays_o,
                           const float* rays_d, uint32_t N, const float* cam_near_far,
                           uint32_t n_cnf, float bg_color, float* image, float* depth,
                           float* weights_sum, float* samvit, float* feature_rows,
                           void* workspace, size_t workspace_bytes, samnerf_stream_t stream);

/* The same render writing every per-ray output into one row-major tile
 * [N, ld] instead of separate arrays: columns 0-2 image, 3 depth, 4
 * weights_sum, 5-260 samvit (feats != 0 and with_sam; ld >= 261, else ld >= 5,
 * the feature columns untouched).  This is the all-gather record of a
 * ray-sharded view (samnerf_amd/dist.py, BASELINE config 4): a rank renders
 * its band straight into its slice of the gather buffer, so no pack copy
 * precedes the collective.  Replaces the reference's per-chunk torch.cat of
 * the outputs (renderer.py:205-217) for that path; bit-identical values. */
int samnerf_render_forward_tile(const samnerf_model* model, const float* rays_o,
                                const float* rays_d, uint32_t N, const float* cam_near_far,
                                uint32_t n_cnf, float bg_color, float* tile, uint32_t ld,
                                int feats, float* feature_rows, void* workspace,
                                size_t workspace_bytes, samnerf_stream_t stream);

/* The SAM head alone (samvit_mlp = SkipConnMLP(163, 256 x 5) + LayerNorm(256),
 * nerf/network.py:36-75, :120-123) on given head-input rows [N,164] (the
 * feature_rows layout of samnerf_render_forward: cat(f_sam, f_image, image,
 * depth) + 1 pad column) -> samvit [N,256], at model->head_mode's precision
 * (0 = f16x3, the default; 1 = exact fp32 MFMA).  The render runs the same
 * kernels on its own rows; this entry point serves callers that hold rows
 * (the reference's samvit_mlp call on a feature batch, renderer.py:384-388). */
size_t samnerf_sam_head_workspace_size(void);
int samnerf_sam_head_forward(const samnerf_model* model, const float* rows, uint32_t N,
                             float* samvit, void* workspace, size_t workspace_bytes,
                             samnerf_stream_t stream);

/* instance_mask_logits [N, mask_out] (renderer.py:392-395, :451-452):
 * sum_k w_k * mask_mlp(cat(m_grid(x_k), geo_feat_k)) over the final samples, the
 * weights and positions those of the samnerf_render_forward call that last used
 * `workspace` (same model, N and view_width; it stores each sample's geo_feat
 * when model->with_mask).  Precision follows head_mode (bf16x3 / exact fp32 MFMA).
 * Replaces the reference's per-chunk torch ops of that branch. */
int samnerf_mask_forward(const samnerf_model* model, uint32_t N, float* instance_mask_logits,
                         const void* workspace, size_t workspace_bytes, samnerf_stream_t stream);

/* The --with_mask training step's instance head (nerf/utils.py:941-977 under
 * renderer.py:392-395, :451-452; 'default' head, network.py:125-133), exact fp32
 * on MFMA.  forward: instance_mask_logits [N, mask_out] from the final samples
 * (positions, weights, geo_feat) that the samnerf_render_forward call with
 * with_mask = 1 left in `render_ws`, saving the head's activations in
 * `workspace` (samnerf_mask_train_workspace_size(N) bytes); backward: given
 * d loss / d logits [N, mask_out], writes the gradients of mask_w[0..2]
 * ([256,143] [256,256] [mask_out,256], overwritten) and scatters into
 * grad_m_grid (the m_grid embedding gradient, accumulated into: the
 * reference encoder's backward).  weights and geo_feat carry no gradient
 * (.detach() in the reference), the sample positions none (no parameter).
 * Replaces the reference's per-chunk torch ops and autograd of that branch.
 * 'adaptive' heads (mask_kind 1 'density', network.py:167-180, the reference's
 * scripts/train_mask.sh:16,20,21 configuration; 2 'rgb' with sum_after_mlp,
 * network.py:148-160): the render leaves each ray's weighted sums of the
 * head's (detached) inputs in `render_ws`; forward runs the bias-free Linear
 * chain on them (the head is linear: the logits of the per-sample chain and
 * weighted sum, to rounding), backward writes the gradients of every
 * mask_w[i] ([96,32] .. [mask_out,96], overwritten, fixed-order sums) -- the
 * only tensors the reference's loss reaches; grad_m_grid is unused (may be
 * NULL).  Workspace (same size function): 2 x 7 x 96 floats per ray. */
/* The 'default' head's workspace keeps its fp32 activations of all 32 samples of every
 * ray for the backward -- input (144), both hidden layers and their
 * gradients (4 x 256) and the logits and their gradient (2 x 32): about 157 KB
 * per ray, 0.64 GB at the reference's 4,096-ray batch (and the render's own
 * workspace stays alive until the backward).  Batches of 65,536 rays need
 * ~10 GB. */
size_t samnerf_mask_train_workspace_size(uint32_t N);
/* The workspace the given mask model needs (what samnerf_mask_train_workspace_size(N)
 * returns is the maximum over the head kinds): the 'default' head's
 * activation carve above, or 2 x 7 x 96 floats per ray for the adaptive heads
 * (mask_kind 1 / 2) -- ~5.4 KB per ray instead of ~157 KB. */
size_t samnerf_mask_train_workspace_size_model(const samnerf_model* model, uint32_t N);
int samnerf_mask_train_forward(const samnerf_model* model, uint32_t N, float* instance_mask_logits,
                               const void* render_ws, size_t render_ws_bytes, void* workspace,
                               size_t workspace_bytes, samnerf_stream_t stream);
int samnerf_mask_train_backward(const samnerf_model* model, uint32_t N, const float* grad_logits,
                                float* const* grad_mask_w, float* grad_m_grid, const void* render_ws,
                                size_t render_ws_bytes, void* workspace, size_t workspace_bytes,
                                samnerf_stream_t stream);

/* Backward of the s_grid feature composite for the SAM-distillation step
 * (nerf/utils.py:1098-1106 training branch): given the per-ray gradient of
 * f_sam [N,128] (the first 128 columns of d(loss)/d(feature_rows)), scatter
 * sum_k w_k * trilinear(corner) * g into grad_embeddings [rows, 8] of s_grid
 * (accumulated into).  Uses the sample weights/positions the last
 * samnerf_render_forward call left in `workspace` for the same rays. */
int samnerf_sgrid_backward(const samnerf_model* model, const float* grad_fsam, uint32_t N,
                           float* grad_embeddings, const void* workspace,
                           size_t workspace_bytes, samnerf_stream_t stream);

/* Deterministic form of samnerf_sgrid_backward (an optional mode
 * whose gradients repeat bit for bit run to run).  The reference scatters
 * with unordered fp32 atomics (gridencoder.cu:334-347), as the default form
 * does, so two identical steps differ in the last bits.  Here every
 * contribution is added to a 64-bit fixed-point accumulator instead (integer
 * atomics are associative: the totals do not depend on the order the waves
 * reach a row in), at the scale 2^(61 - ceil(log2 N) - e) with max |grad_fsam|
 * < 2^e, so no total can overflow and each is resolved to max|g| 2^-(61 -
 * ceil(log2 N)); then the totals are added to grad_embeddings as fp32.
 * accum: accum_bytes >= samnerf_sgrid_accum_size(model) bytes of device
 * memory (else SAMNERF_EWORKSPACE), all zero on the first call (hipMemset)
 * and left zero by every call; one accumulator per stream (calls on one
 * stream run in order; concurrent calls must not share one).  A grad_fsam
 * holding a NaN or an Inf has no fixed-point scale: such a call adds with
 * the fp32 atomics, so the NaN / Inf reaches grad_embeddings as in the
 * reference (bits repeat for finite gradients only). */
size_t samnerf_sgrid_accum_size(const samnerf_model* model);
int samnerf_sgrid_backward_det(const samnerf_model* model, const float* grad_fsam, uint32_t N,
                               float* grad_embeddings, int64_t* accum, size_t accum_bytes,
                               const void* workspace, size_t workspace_bytes,
                               samnerf_stream_t stream);

/* ------------------------------------------------------------- training --
 * One Adam step (torch.optim.Adam semantics, amsgrad off, maximize off) over
 * every tensor of the table in one launch: param -= lr / (1 - beta1^step) *
 * m / (sqrt(v) / sqrt(1 - beta2^step) + eps) after m, v absorb grad (+
 * weight_decay * param).  The optimiser of the distillation step
 * (nerf/utils.py:1831, Adam(lr 1e-2, eps 1e-15) of main.py:296).  Tensors
 * with a NULL grad are skipped (torch skips parameters without .grad); step
 * counts from 1 and is the same for every tensor of the call.  The scalars
 * are doubles (Python floats): derived ones (1 - beta, bias corrections) are
 * formed in double and rounded to float once, as torch does. */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    uint64_t n;                   /* elements */
} samnerf_adam_tensor;
int samnerf_adam_step(const samnerf_adam_tensor* tensors_host, uint32_t n_tensors, double lr,
                      double beta1, double beta2, double eps, double weight_decay, uint32_t step,
                      samnerf_stream_t stream);

/* The SAM head of the distillation step with its backward (nerf/network.py:
 * 36-75, :120-123 under nerf/utils.py:1098-1106), exact fp32 on MFMA.
 * forward: rows [N,164] (the head input rows of samnerf_render_forward's
 * feature_rows) -> samvit [N,256]; saves the activations in `workspace`
 * (samnerf_head_train_workspace_size(N) bytes), which the backward of the
 * same rows reads.  backward: grad_samvit [N,256] -> grad_rows [N,164]
 * (every column written, column 163 -- depth's padding -- as 0), and
 * OVERWRITES grad_w[5] ([256,163], [256,256], [256,419], [256,256],
 * [256,256]), grad_b[5] ([256] each), grad_ln_w, grad_ln_b ([256]); no
 * buffer needs zeroing by the caller.  The weights are the model's sam_w /
 * sam_b / ln_w / ln_b. */
size_t samnerf_head_train_workspace_size(uint32_t N);
int samnerf_head_train_forward(const samnerf_model* model, const float* rows, uint32_t N,
                               float* samvit, void* workspace, size_t workspace_bytes,
                               samnerf_stream_t stream);
int samnerf_head_train_backward(const samnerf_model* model, const float* rows,
                                const float* grad_samvit, uint32_t N, float* grad_rows,
                                float* const* grad_w, float* const* grad_b, float* grad_ln_w,
                                float* grad_ln_b, void* workspace, size_t workspace_bytes,
                                samnerf_stream_t stream);

/* One RGB training step (Trainer.train_step's RGB branch, nerf/utils.py:897-937,
 * over NeRFRenderer.run in train mode, nerf/renderer.py:221-362): the render of
 * N rays (perturbed when model->perturb is set, as the reference trains), the loss
 * MSE(image, gt) + lambda_proposal * proposal_loss (renderer.py:30-57, when
 * update_proposal) + lambda_distort * distort_loss (renderer.py:17-27, the
 * eff_distloss form) + lambda_entropy * entropy(weights_sum) (utils.py:926-929),
 * and its gradient w.r.t. every trained tensor -- what loss.backward() leaves in
 * .grad.  RGB models only (no SAM / mask head, sum_after_mlp off).  fp32.
 *   gt_rgb [N,3] (already composited on the background); image [N,3], depth [N],
 *   weights_sum [N] the render's outputs; loss [5] (device): mse, proposal,
 *   distortion, entropy (the unweighted means) and the total.
 *   Gradients are OVERWRITTEN (zero-filled first); with update_proposal == 0 (or
 *   lambda_proposal == 0) the proposal gradients are not touched and may be NULL
 *   (the reference computes no gradient for them then).
 * Replaces the ~350-op forward and the autograd backward of the torch path. */
typedef struct {
    float lambda_proposal;        /* main.py:106, default 1 */
    float lambda_distort;         /* main.py:108, default 0.02 */
    float lambda_entropy;         /* main.py:100, default 0 */
    int update_proposal;          /* utils.py:912-913 */
    float bg_color;               /* scalar background (1 for 'last_sample') */
} samnerf_rgb_train_opts;
typedef struct {
    float* grid;                  /* grid.embeddings [rows,2] */
    float* grid_mlp[3];           /* [64,32] [64,64] [16,64] */
    float* view_mlp[3];           /* [32,31] [32,32] [3,32] */
    float* prop[2];               /* prop_encoders.{0,1}.embeddings */
    float* prop_mlp[2][2];        /* [16,10] [1,16] each */
} samnerf_rgb_grads;
/* Workspace for N rays of this model: the saved activations plus 8 per-XCD
 * copies of the leading grid levels' gradient rows (those within 600 K rows), so
 * it depends on the model's table offsets as well as on N. */
size_t samnerf_rgb_train_workspace_size(const samnerf_model* model, uint32_t N);
/* The same step as an autograd pair -- NeRFRenderer.run in train mode under
 * grad (renderer.py:221-362), differentiable outputs image, depth, weights_sum and
 * the render's own losses (proposal_loss when with_proposal, distort_loss), the
 * Trainer's criterion left to the caller:
 *   forward: weights [N,32] (or NULL) = the final samples' weights, results['weights']
 *     of renderer.py:350; losses [2] (device) = (proposal_loss,
 *     distort_loss), unweighted; keeps
 *     what the backward reads in `workspace` (same model, rays, N, perturb arrays);
 *   backward: grad_image [N,3], grad_weights_sum [N] / grad_depth [N] / grad_weights
 *     [N,32] (NULL = 0), grad_losses [2] (device; NULL = 0, required with
 *     with_proposal) -> the
 *     gradients, OVERWRITTEN as in samnerf_rgb_train_step. */
int samnerf_rgb_train_forward(const samnerf_model* model, const float* rays_o, const float* rays_d,
                              uint32_t N, const float* cam_near_far, uint32_t n_cnf, float bg_color,
                              int with_proposal, float* image, float* depth, float* weights_sum,
                              float* weights, float* losses, void* workspace, size_t workspace_bytes,
                              samnerf_stream_t stream);
int samnerf_rgb_train_backward(const samnerf_model* model, const float* rays_o, const float* rays_d,
                               uint32_t N, float bg_color, int with_proposal, const float* grad_image,
                               const float* grad_weights_sum, const float* grad_depth,
                               const float* grad_weights, const float* grad_losses,
                               const samnerf_rgb_grads* grads, void* workspace, size_t workspace_bytes,
                               samnerf_stream_t stream);
int samnerf_rgb_train_step(const samnerf_model* model, const float* rays_o, const float* rays_d,
                           uint32_t N, const float* cam_near_far, uint32_t n_cnf, const float* gt_rgb,
                           const samnerf_rgb_train_opts* opts, float* image, float* depth,
                           float* weights_sum, float* loss, const samnerf_rgb_grads* grads,
                           void* workspace, size_t workspace_bytes, samnerf_stream_t stream);

/* Transport record of the per-ray outputs for the all-gather of a
 * ray-sharded view (samnerf_amd/dist.py; no reference counterpart: the
 * reference renders on one GPU, nerf/renderer.py:185-219).  One record of
 * samnerf_tile_words() 32-bit words per ray: image[3], depth, weights_sum
 * (fp32, exact), a power-of-two scale s and samvit[256] as int16 q = rint(v/s)
 * (|v - q s| <= 2^-14 of the ray's max |samvit|; NaN / inf rays decode to NaN).
 * samvit must be 16-B aligned, tile 8-B aligned; N = 0 is a no-op. */
uint32_t samnerf_tile_words(void);
int samnerf_tile_encode(const float* image, const float* depth, const float* weights_sum,
                        const float* samvit, uint32_t N, void* tile, samnerf_stream_t stream);
int samnerf_tile_decode(const void* tile, uint32_t N, float* image, float* depth,
                        float* weights_sum, float* samvit, samnerf_stream_t stream);

/* Parity taps (tests only; no reference counterpart -- they expose what
 * nerf/renderer.py:261-326 and network.py:221-259 compute between its ops).
 * While set, every samnerf_render_forward call of this thread over exactly N
 * rays writes the stages' intermediates to these device buffers as well (the
 * same kernels run, with one predicated store per tapped value; outputs are
 * unchanged; rays are not regrouped into pixel tiles), sample-major:
 *   ds0 [128][N], ds1 [64][N]   optical depth delta * sigma of each proposal
 *                               sample (renderer.py:310-311)
 *   w0 [128][N], w1 [64][N]     their composited weights (renderer.py:312-326),
 *                               the input of sample_pdf
 *   bins1 [65][N], bins2 [33][N]  the resampled bins of sample_pdf
 *                               (renderer.py:274-275)
 *   inds1 [65][N], inds2 [33][N]  its torch.searchsorted(cdf, u, right=True)
 *                               indices (renderer.py:105), int32
 *   sigma2 [32][N]              the final stage's sigma = trunc_exp(density)
 *                               of every sample (network.py:227, k_final)
 *   w2 [32][N]                  the final stage's composited weights
 *                               (renderer.py:312-326)
 *   u2 [32][3][N]               the final samples' grid-space positions
 *                               (contract(xyz) + bound) / (2 bound), grid.py:156
 *   rows2, srows [ceil(N / row_stride)][32][16][8]  uint32, for the rays
 *                               r % row_stride == 0: the level-relative corner
 *                               row each trilinear weight multiplies, per final
 *                               sample, level and corner (bit 0 x, 1 y, 2 z, as
 *                               gridencoder.cu:61-79): rows2 those of k_final's
 *                               grid gathers, srows those of the s_grid
 *                               composite (k_sgrid_box4, N >= 32768 only;
 *                               samples whose weight is 0 on all 64 rays of a
 *                               wave are skipped and left unwritten)
 * Any pointer may be NULL.  taps = NULL clears them; a render over another
 * ray count fails with SAMNERF_EINVAL while they are set.  Thread-local. */
typedef struct {
    float* ds0;
    float* ds1;
    float* w0;
    float* w1;
    float* bins1;
    float* bins2;
    int32_t* inds1;
    int32_t* inds2;
    float* sigma2;
    float* w2;
    float* u2;
    uint32_t row_stride;
    uint32_t* rows2;
    uint32_t* srows;
} samnerf_taps;
int samnerf_set_taps(const samnerf_taps* taps, uint32_t N);

/* Measurement hook (bench.py): when set, samnerf_render_forward records
 * events[i] (hipEvent_t) on its stream before stage i (0 prop0, 1 prop1,
 * 2 final, 3 s_grid, 4 SAM head) and events[5] after the last one.  n = 0 or
 * events = NULL disables it.  Thread-local; costs one hipEventRecord per stage. */
int samnerf_set_stage_events(void* const* events, uint32_t n);

/* Test hook: the compiled kernel forms the last samnerf_render_forward(_tile)
 * of this thread launched, so the tests can tell which specialisation ran.
 * out[0] / out[1]: the proposal stages' level classes (dense-level mask |
 * hashed-level mask << 8) when k_prop_sigma ran with them as compile-time
 * constants, 0 for the run-time form; out[2]: k_final's layout (1 = the
 * reference grid's compile-time slot layout, 0 = run-time); out[3] reserved.
 * Writes min(n, 4) entries, returns 4.  Thread-local, no GPU work. */
int samnerf_last_forms(uint32_t* out, uint32_t n);

/* Measurement hook (bench.py): one stamp of the shader clock on `stream`,
 * from 256 single-wave workgroups (every XCD): out[3 * b + 0] = XCC id,
 * out[3 * b + 1] = s_memtime (shader-clock ticks), out[3 * b + 2] =
 * s_memrealtime (100 MHz) of workgroup b; out holds 768 uint64.  Two stamps
 * around the timed views give the clock they ran at per XCD:
 * d(memtime) / d(memrealtime) x 100 MHz.  Costs one ~5-us launch. */
int samnerf_clock_stamp(uint64_t* out, samnerf_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* SAMNERF_HIP_H */
