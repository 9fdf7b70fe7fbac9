/* espnet_mi355.h — C ABI of libespnet_mi355.so, the MI355X (gfx950) kernels behind
 * espnet_slurp_amd's drop-in ESPnet2 ASR training step.
 *
 * Conventions (every entry point):
 *   - plain device pointers (fp32 unless stated; int64 token ids as `long long`), sizes as int/long;
 *   - row-major, the layouts documented per function;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued asynchronously, nothing syncs;
 *   - return 0 on success, non-zero on a launch/argument error; esp_last_error() describes it
 *     (thread-local).  No allocation happens inside: callers pass workspaces.
 *
 * Which reference interface each entry point replaces (BriansIDP/espnet_slurp, file:line):
 *   the reference has no native code on this path; these functions replace
 *   the ATen ops its Python building blocks call.  The reference-side "binding" is the espnet2
 *   plugin registry (espnet2/tasks/asr.py:133-188); see INTEGRATION.md.
 */
#ifndef ESPNET_MI355_H
#define ESPNET_MI355_H
#ifdef __cplusplus
extern "C" {
#endif

const char* esp_last_error(void);
int esp_abi_version(void);

/* ---- MFMA GEMM (nn.Linear fwd/bwd, Conv1d k=1, Conv2d via implicit im2col, attention
 * matmuls; attention.py:55-58,112,200-205, positionwise_feed_forward.py:32,
 * convolution.py:70-77, subsampling.py:84-85).
 *   C[z](m,n) = alpha*epi(sum_k A(m,k) B(k,n) + bias[n]) + beta*R[z](m,n)
 *   mode 0 (KC): elem(r,k)=p[r*ld+k]   mode 1 (RC): elem(r,k)=p[k*ld+r]
 *   mode 2/3: im2col of an NHWC map (3x3, stride 2); im2col_x = {H, W, C, Ho, Wo}
 *   z = z1*nb2+z2 ; operand offset = z1*s1 + z2*s2
 *   act: 0 none, 1 ReLU, 2 Swish (pre-activation stored to aux if non-NULL); dropout with
 *   probability drop_p keyed by (seed, (z*M+m)*N+n).  Every dropout site of this ABI rounds
 *   drop_p to the nearest multiple of 1/65536 (at least 1/65536 when drop_p > 0: a positive p
 *   never turns dropout off) and scales kept values by 1 / (1 - rounded p), so E[out] = in.
 *   bwd_act != 0 (backward of h = drop(act(pre)), positionwise_feed_forward.py:32): the
 *   epilogue is  v = drop'(acc + bias) * act'(pre)  with the dropout mask regenerated from
 *   (drop_p, seed); act must be 0 and aux NULL.
 *   rowsum != NULL (mode_a RC, batch 1): rowsum[m] += sum_k A(m,k) — the bias gradient of a
 *   weight-gradient GEMM (dW = dy^T x, db = colsum dy) in the same pass over dy.
 *   work/work_bytes: optional scratch; when the tile grid is too small to fill the chip the
 *   K range is split over blocks and reduced (fixed order, deterministic) before the epilogue.
 *   The last 64 KiB of work (work_bytes > 64 KiB) hold the split-K arrival tickets of the
 *   in-kernel combine: the caller zero-fills them once before the first call that uses this
 *   workspace and every launch leaves them zero; one workspace must not serve two launches
 *   that run concurrently (e.g. on two streams). */
int esp_gemm_f32(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2,
                 const float* A, long lda, long sa1, long sa2,
                 const float* B, long ldb, long sb1, long sb2,
                 float* C, long ldc, long sc1, long sc2,
                 const float* bias, float alpha, float beta, const float* R,
                 int act, float* aux, float drop_p, unsigned long long seed,
                 int bwd_act, const float* pre, float* rowsum,
                 const int* im2col_a, const int* im2col_b, float* work, long work_bytes,
                 void* stream);
/* GEMM compute type for every later esp_gemm_f32 launch (process-wide host state, read at
 * launch time, so a captured HIP graph keeps the kernels of its capture): 0 = fp32 MFMA
 * (default; the reference's train_dtype float32), 1 = bf16 operands (fp32 values rounded to
 * nearest-even while staged into LDS) with fp32 accumulate and fp32 epilogue / outputs.
 * Mode 1 is the reduced-precision training path of SURVEY §8(d) C5; the reference's nearest
 * knob is `use_amp` (fp16 autocast, trainer.py:181-195,554).  Returns the previous value. */
int esp_set_gemm_compute(int dtype);
int esp_get_gemm_compute(void);
/* How the fp32 compute type (0) multiplies in the LDS-DMA GEMM kernel of this build: 6 = each
 * fp32 operand split exactly into three bf16 (hi + mid + lo, round-to-nearest-even residuals)
 * and the six products down to 2^-16 relative (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid)
 * accumulated in fp32 on v_mfma_f32_32x32x16_bf16 (the dropped terms are <= 2^-23 |a b|, below
 * an fp32 rounding of the sum); 1 = v_mfma_f32_32x32x2_f32 (build flag ESP_F32_SPLIT=0). */
int esp_f32_gemm_products(void);
/* Split-K combine of every later esp_gemm_f32 launch (process-wide): 0 = a separate
 * fixed-order reduction launch (default), 1 = in-kernel (the last-arriving unit of each output
 * tile sums the splits in fixed order; needs the zeroed ticket area of `work`, see above).
 * Initialised from ESP_SPLITK_INKERNEL.  Returns the previous mode. */
int esp_set_splitk_mode(int mode);
/* esp_gemm_f32 with B also given as its three bf16 split planes (esp_f32_to_planes of the fp32 B,
 * b = hi + mid + lo exactly): the same fp32 split products as esp_gemm_f32 on the fp32 B, in the same
 * order, bit for bit (split-K counts may differ: a different tile width), without splitting B in the
 * GEMM's k-loop.  b_planes: plane 0; plane p at b_planes + p * b_pstride bf16 elements; ldbp, sbp1,
 * sbp2 in bf16 elements.  Used when the fp32 compute type is active, mode_b is KC or RC and the planes
 * qualify (16-B aligned, ldbp / strides / pstride % 8 == 0, K % 8 == 0 for KC, N % 8 == 0 for RC);
 * otherwise -- or when the epilogue kind has no B-planes kernel -- the fp32 B (which may then not
 * be NULL) is used.  Reference: every nn.Linear / Conv weight operand of the step (weights are
 * split once per step, kernels.py). */
int esp_gemm_f32_bp(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                    long sa1, long sa2, const float* B, long ldb, long sb1, long sb2, float* C, long ldc,
                    long sc1, long sc2, const float* bias, float alpha, float beta, const float* R, int act,
                    float* aux, float drop_p, unsigned long long seed, int bwd_act, const float* pre, float* rowsum,
                    const int* im2col_a, float* work, long work_bytes, const void* b_planes, long ldbp, long sbp1,
                    long sbp2, long b_pstride, void* stream);
/* esp_gemm_f32 with either operand, or both, also given as its three bf16 split planes (layout of
 * esp_gemm_f32_bp's B planes; A planes: a_planes, ldap, sap1, sap2, a_pstride in bf16 elements, mode KC
 * or RC, K % 8 == 0 for KC, M % 8 == 0 for RC).  Both as planes: no operand split in the k-loop (the
 * same products, bit for bit; 64-wide tiles).  An operand whose planes do not qualify, or a launch
 * with no planes kernel, takes its fp32 values (which may then not be NULL); A NULL fp32 operand with
 * qualifying planes is allowed.  mode_a, mode_b: 0 (KC) or 1 (RC).
 * c_nplanes 3 or 1: C is written as bf16 planes (the exact split / bf16) instead of fp32 -- C points at
 * plane 0, plane p at C + p * c_pstride bf16 elements, ldc / sc1 / sc2 in bf16 elements (aux and pre
 * share those offsets in fp32 elements) -- for the epilogues whose result only GEMMs read: plain
 * (the attention context), bias + activation + dropout + derivative (the FFN hidden state) and the
 * backward multiply by pre (bwd_act ACT_MUL, no dropout / bias: the FFN hidden-state gradient);
 * N % 4 == 0, no residual, no row sums, never split-K.  0: fp32 C. */
int esp_gemm_f32_pl(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const float* A, long lda,
                    long sa1, long sa2, const void* a_planes, long ldap, long sap1, long sap2, long a_pstride,
                    const float* B, long ldb, long sb1, long sb2, const void* b_planes, long ldbp, long sbp1,
                    long sbp2, long b_pstride, float* C, long ldc, long sc1, long sc2, const float* bias,
                    float alpha, float beta, const float* R, int act, float* aux, float drop_p,
                    unsigned long long seed, int bwd_act, const float* pre, float* rowsum, int c_nplanes,
                    long c_pstride, float* work, long work_bytes, void* stream);
/* The three bf16 planes of a rows x cols fp32 matrix x (row pitch ldx): plane p at y + p * pstride
 * (bf16 elements, row pitch ldy), hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid), round to
 * nearest even with exact fp32 residuals, so x = hi + mid + lo for every finite x.  Columns
 * cols..ldy-1 are written 0.  ldy, pstride % 8 == 0, pstride >= rows * ldy, y 16-B aligned. */
int esp_f32_to_planes(const float* x, void* y, long rows, int cols, long ldx, long ldy, long pstride, void* stream);
/* bf16-operand GEMM (the C5 reduced-precision path): A and B bf16 (bits of __bf16 /
 * torch.bfloat16) in mode KC or RC as esp_gemm_f32 (KC: [rows][K]; RC: [K][rows], staged for
 * transposing LDS reads), fp32 accumulate; C, the epilogue (bias, act, aux, dropout, bwd_act /
 * pre, residual) and split-K exactly as esp_gemm_f32.  K, lda, ldb and the batch strides in bf16
 * elements, multiples of 8; A, B 16-B aligned; an RC operand's row count a multiple of 8.
 * rowsum != NULL (mode_a RC, batch 1): rowsum[m] += sum_k A(m,k) in fp32 over the bf16 values.  The
 * operands come from esp_f32_to_bf16 (activations, gradients) or bf16 weight copies. */
int esp_gemm_bf16(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const void* A, long lda,
                  long sa1, long sa2, const void* B, long ldb, long sb1, long sb2, float* C, long ldc,
                  long sc1, long sc2, const float* bias, float alpha, float beta, const float* R, int act,
                  float* aux, float drop_p, unsigned long long seed, int bwd_act, const float* pre, float* rowsum,
                  float* work, long work_bytes, void* stream);
/* esp_gemm_bf16 with C written as its bf16 plane (c_nplanes 1: hi = bf16(C), the reduced-precision
 * path's GEMM-only activations and gradients) under the rules of esp_gemm_f32_pl's c_nplanes: the
 * plain, FFN w_1 and ACT_MUL epilogues, N % 4 == 0, no residual / row sums, never split-K. */
/* The bf16 mode's conv2 forward (subsampling.py:53-87, NHWC): z2 = ReLU(im2col(z1_16) w16^T + bias) on
 * bf16 operands (z1_16 from esp_conv1_fwd_bf16, w16 the (o, kt, kf, c)-laid weights in bf16, row pitch
 * 9D), fp32 accumulate and output.  D % 64 == 0, 16-B aligned operands. */
int esp_conv2_fwd_bf16(const void* z1_16, const void* w16, const float* bias, float* z2, int B, int T1, int F1, int D,
                       float* work, long work_bytes, void* stream);
/* The bf16 mode's conv2 weight gradient: dw (D x 9D, (o, kt, kf, c) order) = dz2^T im2col(z1) and
 * db += column sums of dz2, on bf16 operands (dz2_16 [pixels][D], z1_16 from esp_conv1_fwd_bf16); an
 * even pixel count, D % 64 == 0, 16-B aligned; `work` the split-K partials as esp_gemm_f32's. */
int esp_conv2_wgrad_bf16(const void* dz2_16, const void* z1_16, float* dw, float* db, int B, int T1, int F1, int D,
                         float* work, long work_bytes, void* stream);
/* esp_conv2_dgrad with dz2 in bf16 (the bf16 mode): the class GEMMs on bf16 operands (workspace as
 * esp_conv2_dgrad's).  D % 64 == 0. */
int esp_conv2_dgrad_bf16(const void* dz2_16, const float* W, const float* z1, float* dz1, int B, int T1, int F1, int D,
                         const float* zeros16, float* wc_work, long work_bytes, void* stream);
int esp_gemm_bf16_pl(int mode_a, int mode_b, int M, int N, int K, int batch, int nb2, const void* A, long lda,
                     long sa1, long sa2, const void* B, long ldb, long sb1, long sb2, void* C, long ldc,
                     long sc1, long sc2, const float* bias, float alpha, float beta, int act, float* aux,
                     float drop_p, unsigned long long seed, int bwd_act, const float* pre, int c_nplanes,
                     long c_pstride, float* work, long work_bytes, void* stream);
/* y = bf16(x) (round to nearest even) for a rows x cols fp32 matrix (row pitch ldx); transpose:
 * y[c * ldy + r] (a cols x rows bf16 matrix), else y[r * ldy + c]. */
int esp_f32_to_bf16(const float* x, void* y, long rows, int cols, long ldx, long ldy, int transpose,
                    void* stream);

/* ---- element-wise (positionwise_feed_forward.py:32, conformer/swish.py:13-18, dropout) */
int esp_act_bwd(const float* dy, const float* h, float* dx, long n, int act, float drop_p,
                unsigned long long seed, long idx_off, void* stream);
int esp_scale_dropout(const float* x, float* y, long n, float alpha, float drop_p,
                      unsigned long long seed, const float* r, float beta, void* stream);
/* y = alpha * drop(x) written as bf16 planes (nplanes 3 exact split, 1 bf16; plane p at y + p * pstride
 * bf16 elements) of a matrix with ld == cols (n = rows * cols, % 4 == 0): the same masks as
 * esp_scale_dropout for the same (drop_p, seed). */
int esp_scale_dropout_planes(const float* x, void* y, long n, long pstride, int nplanes, float alpha, float drop_p,
                             unsigned long long seed, void* stream);
int esp_scale_by_dev(float* x, long n, const float* s, void* stream);
/* decoder embedding + abs positional encoding (transformer_decoder.py:68-71, embedding.py:81-94) */
int esp_embed_fwd(const long long* tok, const float* E, const float* pe, float* y, int nrows, int L,
                  int D, float xscale, float drop_p, unsigned long long seed, void* stream);
int esp_embed_bwd(const long long* tok, const float* dy, float* dE, int nrows, int V, int D,
                  float xscale, float drop_p, unsigned long long seed, void* stream);
/* SpecAug with injected draws (specaug.py:89-96, time_warp.py:9-88, mask_along_axis.py:8-68):
 * lens (B) int32; warp (B,2) {center, warped} or NULL (center<=0: no warp for that row);
 * fmask (B,nf,2) / tmask (B,nt,2) {pos, width}. */
int esp_specaug(const float* x, float* y, int B, int T, int F, const int* lens, const int* warp,
                const int* fmask, int nf, const int* tmask, int nt, void* stream);
/* UtteranceMVN(norm_means=True, norm_vars=False), in place (utterance_mvn.py:45-80) */
int esp_utterance_mvn(float* x, int B, int T, int F, const int* lens, void* stream);
/* clip_grad_norm_ + Adam over flat buffers (trainer.py:642-686, abs_task.py:78-79) */
int esp_grad_norm(const float* g, long n, float max_norm, double* work, long work_bytes, float* out3,
                  void* stream);
int esp_adam(float* p, const float* g, float* m, float* v, long n, const float* clip3, float lr,
             double b1, double b2, float eps, float wd, int step, void* stream);
/* Device-resident optimizer bookkeeping (a whole training step as one HIP graph):
 * state (2 doubles) = {Adam steps applied, WarmupLR steps taken}.  esp_opt_hyper writes the
 * next step's {lr, 1-b1^t, sqrt(1-b2^t)} (warmuplr.py:43-50, torch Adam) to hyper (3 floats);
 * esp_adam_dev reads them; esp_opt_advance counts the step only if clip3[2] (finite) != 0,
 * which is exactly when trainer.py:651-686 steps the optimizer and the scheduler. */
int esp_opt_hyper(const double* state, double base_lr, double warmup, double b1, double b2, float* hyper,
                  void* stream);
int esp_adam_dev(float* p, const float* g, float* m, float* v, long n, const float* clip3,
                 const float* hyper, double b1, double b2, float eps, float wd, void* stream);
int esp_opt_advance(double* state, const float* clip3, void* stream);
/* ABI 30: torch.optim.Adam(amsgrad=True) (the optim_conf key abs_task.py:856-880 passes through): as
 * esp_adam / esp_adam_dev, the denominator on vmax = max(vmax, exp_avg_sq), kept in place (n floats).
 * ABI 30 also passes beta1 / beta2 of every Adam entry as double: 1 - beta and the bias corrections are
 * formed in double as torch forms them from python floats (fp32 1 - 0.999f is 1.3e-5 off 0.001). */
int esp_adam_amsgrad(float* p, const float* g, float* m, float* v, float* vmax, long n, const float* clip3,
                     float lr, double b1, double b2, float eps, float wd, int step, void* stream);
int esp_adam_dev_amsgrad(float* p, const float* g, float* m, float* v, float* vmax, long n, const float* clip3,
                         const float* hyper, double b1, double b2, float eps, float wd, void* stream);
/* Dropout key: every dropout kernel XORs its seed with *key when set (NULL: off).  The key
 * lives in device memory so a replayed HIP graph draws fresh masks; esp_rng_advance mixes it
 * (splitmix64) on device. */
int esp_set_rng_key(const unsigned long long* key);
int esp_rng_advance(unsigned long long* key, void* stream);

/* ---- normalisation (layer_norm.py:12-38; convolution.py:56-79) */
int esp_layernorm_fwd(const float* x, const float* w, const float* b, float* y, float* mean,
                      float* rstd, int M, int D, float eps, void* stream);
/* esp_layernorm_fwd with y written as bf16 planes for GEMM readers (kernels.Planes): nplanes 3 = the
 * exact split hi + mid + lo (esp_f32_to_planes), 1 = bf16(y); plane p at y + p * pstride (bf16
 * elements), row pitch ldy (>= D, % 4 == 0).  D % 4 == 0, x / w / b 16-B aligned, y 8-B aligned. */
int esp_layernorm_fwd_planes(const float* x, const float* w, const float* b, void* y, long ldy, long pstride,
                             int nplanes, float* mean, float* rstd, int M, int D, float eps, void* stream);
/* ABI 29: y written in fp32 (yf, row pitch D, 16-B aligned) AND as planes (as esp_layernorm_fwd_planes):
 * the fp32 mode's LayerNorm outputs that feed a Linear's forward (fp32 A) and its weight gradient (the
 * planes as B, gemm_kernels.h PREC 3).  Replaces the same LayerNorm as esp_layernorm_fwd (layer_norm.py:12-38). */
int esp_layernorm_fwd_dual(const float* x, const float* w, const float* b, float* yf, void* y, long ldy,
                           long pstride, int nplanes, float* mean, float* rstd, int M, int D, float eps,
                           void* stream);
int esp_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean,
                      const float* rstd, float* dx, int accumulate, float* dw, float* db, int M,
                      int D, float* work, long work_bytes, void* stream);
int esp_colsum(const float* x, int M, int N, long ld, float* out, int accumulate, float* work,
               long work_bytes, void* stream);
int esp_glu_fwd(const float* u, float* g, long rows, int D, void* stream);
int esp_glu_bwd(const float* u, const float* dg, float* du, long rows, int D, void* stream);
/* esp_glu_bwd with du written as bf16 planes (nplanes 3 exact split, 1 bf16; row pitch 2D, plane p at
 * du + p * pstride bf16 elements) for pointwise_conv1's gradient GEMMs; D % 4 == 0. */
int esp_glu_bwd_planes(const float* u, const float* dg, void* du, long pstride, int nplanes, long rows, int D,
                       void* stream);
/* tvalid (device int, nullable): the batch is padded to T frames per utterance but only the
 * first *tvalid exist in the reference batch (length-bucketed HIP graphs).  The depthwise
 * convolution reads frames >= *tvalid as its zero padding and writes 0 there; BatchNorm
 * statistics count B * (*tvalid) rows and the excluded rows get a zero gradient.  With tvalid,
 * M = B * T rows for the BatchNorm calls.  BatchNorm workspaces: D * 1536 (forward) and
 * 2 * D * 1536 (backward) doubles — the statistics are reduced in at most 1536 row chunks. */
int esp_dwconv1d(const float* x, const float* W, const float* bias, float* y, int Bn, int T, int D,
                 int K, int flip, const int* tvalid, void* stream);
int esp_dwconv1d_wgrad(const float* dy, const float* x, float* dW, int Bn, int T, int D, int K,
                       float* work, long work_bytes, const int* tvalid, void* stream);
int esp_bn_swish_fwd(const float* y, const float* gamma, const float* beta, float* s, float* mean,
                     float* rstd, float* run_mean, float* run_var, float momentum, float eps, int M,
                     int D, double* work, long work_bytes, int T, const int* tvalid, void* stream);
/* esp_bn_swish_fwd with s written as bf16 planes for pointwise_conv2, its only reader (nplanes 3:
 * the exact split, 1: bf16; plane p at s_planes + p * pstride bf16 elements, row pitch lds).
 * D, lds, pstride % 4 == 0; 16-B aligned y / gamma / beta, 8-B aligned planes. */
int esp_bn_swish_fwd_planes(const float* y, const float* gamma, const float* beta, void* s_planes, long lds,
                            long pstride, int nplanes, float* mean, float* rstd, float* run_mean, float* run_var,
                            float momentum, float eps, int M, int D, double* work, long work_bytes, int T,
                            const int* tvalid, void* stream);
/* eval mode: statistics from run_mean / run_var (mean / rstd written for inspection) */
int esp_bn_swish_eval(const float* y, const float* gamma, const float* beta, float* s, const float* run_mean,
                      const float* run_var, float eps, int M, int D, float* mean, float* rstd, void* stream);
int esp_bn_swish_bwd(const float* ds, const float* y, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, float* dy, float* dgamma, float* dbeta,
                     int M, int D, double* work, long work_bytes, float* sums, int T, const int* tvalid,
                     void* stream);

/* ---- attention glue (attention.py:64-96,145-165,240-263) */
int esp_heads_split(const float* src, long ld, int col0, int B, int T, int H, int dk,
                    const float* bias, float* dst, void* stream);
/* both head-major splits of esp_heads_split in one pass: dst_a = q + bias_a, dst_b = q + bias_b
 * (q + pos_bias_u, q + pos_bias_v; attention.py:240-250).  16-B aligned, dk, ld, col0 % 4 == 0. */
int esp_heads_split2(const float* src, long ld, int col0, int B, int T, int H, int dk, const float* bias_a,
                     float* dst_a, const float* bias_b, float* dst_b, void* stream);
int esp_add2d(const float* x, long ldx, float* y, long ldy, int M, int N, void* stream);
/* score rows (ac / attn / pdrop / dP / dS) have pitch lds >= Tk, bd / dbd rows pitch ldp >= P
 * (multiples of 4 keep every row 16-B aligned for the GEMMs' LDS-DMA staging); dropout
 * masks are keyed by the logical index row*Tk + j, independent of the pitch. */
int esp_attn_softmax_fwd(const float* ac, const float* bd, int relpos, int P, float sqrt_dk,
                         const int* klen, int nb, int causal, float* attn, float* pdrop,
                         float drop_p, unsigned long long seed, int Z, int Tq, int Tk, long lds,
                         long ldp, const int* tvalid, void* stream);  /* tvalid: legacy length bucket, see below */
int esp_attn_softmax_bwd(const float* attn, const float* dP, float* dS, float drop_p,
                         unsigned long long seed, float sqrt_dk, long rows, int Tk, long lds,
                         void* stream);
int esp_relshift_bwd(const float* dS, long lds, float* dbd, long ldp, int relpos, int Z, int T, int P,
                     void* stream);
/* esp_attn_softmax_bwd fused with esp_relshift_bwd (relpos 1 latest: P = 2T-1 columns; relpos 2
 * legacy: P = T columns): writes dS and every dbd element of the rows (pitch ldp) in one pass.
 * rows = Z*T. */
int esp_attn_softmax_bwd_relpos(const float* attn, const float* dP, float* dS, float* dbd, long ldp,
                                int relpos, float drop_p, unsigned long long seed, float sqrt_dk,
                                long rows, int T, long lds, const int* tvalid, void* stream);
/* ABI 29: the latest rel_shift's q_v gradient through the band scores, dq_v[z] = dbd[z] . p_h (z = h*nb + b):
 * the dbd.p contraction with each 128-row tile's k-loop over its rows' band union only (row i of dbd is 0
 * outside columns T-1-i .. 2T-2-i).  dbd (nb*H*T rows, pitch ldp >= 2T-1, % 4 == 0), p (2T-1 rows, pitch
 * ldpm, head h at column 64 h), out rows b*T + i (pitch ldo, head h at column 64 h); d_k = 64. */
int esp_relpos_dqv(const float* dbd, long ldp, const float* p, long ldpm, float* out, long ldo, int nb, int H,
                   int T, float* work, long work_bytes, void* stream);
/* ABI 29: the latest form (P = 2T-1) writing only row i's band of dbd, columns T-1-i .. 2T-2-i, into a
 * buffer whose other elements are already 0 (kept and zeroed once by the caller: nothing else writes it);
 * half the dbd bytes of esp_attn_softmax_bwd_relpos.  lds % 4 == 0, attn / dP / dS 16-B aligned. */
int esp_attn_softmax_bwd_relpos_band(const float* attn, const float* dP, float* dS, float* dbd, long ldp,
                                     float drop_p, unsigned long long seed, float sqrt_dk, long rows, int T,
                                     long lds, void* stream);
/* Fused latest rel-pos attention backward: dP = dctx V^T on the MFMA per 32-row block, attention
 * dropout adjoint, softmax adjoint, rel_shift adjoint -> dS (pitch lds) and dbd (pitch ldp).
 * dctx rows at dctx + (b*T+i)*ldd + 64h, V rows at vmat + (b*T+j)*ldv + 64h; d_k = 64, T <= 512. */
int esp_relpos_attn_bwd(const float* dctx, long ldd, const float* vmat, long ldv, const float* attn,
                        float* dS, float* dbd, long ldp, int nb, int H, float sqrt_dk, float drop_p,
                        unsigned long long seed, int T, long lds, void* stream);
/* Flash-style rel-pos self-attention (csrc/flash_relpos.hip), replacing attention.py:64-96 with
 * the latest (rel = 1, attention.py:240-263, P = 2T-1 position rows) or legacy (rel = 2,
 * attention.py:145-165 rel_shift, P = T rows) score assembly; d_k = 64, T <= 512.
 * q_u = q + pos_bias_u, q_v = q + pos_bias_v: (Z, T, 64) head-major, z = h*nb + b.  k / v rows at
 * kmat + (b*T + j)*ldk + 64h (vmat / ldv alike), p rows at p + row*ldp_row + 64h.
 * Forward: ctx (rows b*T + i, pitch ldc, head slice 64h) = dropout(softmax(s)) v, and the row
 * statistics stats (Z, T, 2) = {max, 1/sum} the backward recomputes P from.  No (Z,T,T) tensor. */
int esp_relpos_flash_fwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* vmat,
                         long ldv, const float* p, long ldp_row, int rel, int nb, int H, float sqrt_dk,
                         const int* klen, float* ctx, long ldc, float* stats, float drop_p,
                         unsigned long long seed, int T, void* stream);
/* Backward of esp_relpos_flash_fwd: recomputes the scores, writes dq (= dq_u + dq_v, rows b*T + i,
 * pitch ldq, head slice 64h; overwritten), dS = dL/d(ac + bd) and the dropped probabilities
 * pdrop (Z, T, lds) for the key-side GEMMs dK = dS^T q_u and dV = pdrop^T dctx, the per-block
 * pos_bias column sums bias_part (Z, ceil(T/32), 2, 64) and, for legacy, carry (Z, ceil(T/32), 64).
 * ctx / dctx: the forward output and its gradient (pitch ldc). */
int esp_relpos_flash_bwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* vmat,
                         long ldv, const float* p, long ldp_row, int rel, int nb, int H, float sqrt_dk,
                         const int* klen, const float* ctx, const float* dctx, long ldc, const float* stats,
                         float drop_p, unsigned long long seed, int T, float* dq, long ldq, float* dS,
                         float* pdrop, long lds, float* bias_part, float* carry, void* stream);
/* linear_pos gradient input from dS and q_v: dp (P x 64H, pitch ldp; overwritten) =
 * sum_{b,i} dbd^T q_v with the rel_shift adjoint read along the diagonals of dS (no dbd tensor);
 * pos_bias_u / pos_bias_v gradients += the column sums of esp_relpos_flash_bwd (du, dv: H x 64);
 * legacy: adds each block's carry to dq (pitch ldq).  work: >= H * ceil(nb/8) * (2T-1) * 64 floats. */
int esp_relpos_dp(const float* dS, long lds, const float* qv, int rel, int nb, int H, int T, float* dp, long ldp,
                  const float* bias_part, const float* carry, float* du, float* dv, float* dq, long ldq,
                  float* work, long work_floats, void* stream);
/* Fused latest rel-pos scores + softmax (attention.py:240-263 with the latest rel_shift,
 * embedding.py:173-244): bd_shift[i][j] = q_v[i] . p[j + T-1-i] is computed on the MFMA per
 * 32-row block inside the kernel (no (Z,T,2T-1) bd tensor), then s = (ac + bd_shift)/sqrt(dk),
 * key mask j < klen[b], softmax, dropout copy.  q_v (Z,T,64) head-major z = h*nb + b;
 * p: P = 2T-1 rows of pitch ldp_row, head h at column 64h.  d_k must be 64; T such that the
 * 32 x (32*ceil((T+31)/32)+4) float window fits 64 KB (T <= 449).  attn may alias ac. */
int esp_relpos_softmax_fwd(const float* qv, const float* p, long ldp_row, int nb, int H, const float* ac,
                           float sqrt_dk, const int* klen, float* attn, float* pdrop, float drop_p,
                           unsigned long long seed, int T, long lds, void* stream);
/* Fully fused latest rel-pos attention probabilities: ac = (q+u) k^T AND the bd band on the
 * MFMA per 32-row block, softmax, dropout copy (attention.py:240-263, 64-96): no score
 * tensor other than attn / pdrop reaches HBM.  q_u, q_v (Z,T,64) head-major z = h*nb + b;
 * k row j of utterance b, head h at kmat + (b*T + j)*ldk + 64h (the fused qkv projection);
 * p as above.  Same limits as esp_relpos_softmax_fwd. */
int esp_relpos_attn_fwd(const float* qu, const float* qv, const float* kmat, long ldk, const float* p,
                        long ldp_row, int nb, int H, float sqrt_dk, const int* klen, float* attn,
                        float* pdrop, float drop_p, unsigned long long seed, int T, long lds,
                        void* stream);
/* Rel-pos attention backward without the (Z,T,T) dP tensor (FlashAttention-2's row term):
 * esp_attn_bwd_prep: dot[z*T+i] = dctx_i . ctx_i per head (= sum_j P_drop[i][j] dP[i][j]) and
 * the bd-gradient elements without a rel_shift source zeroed; esp_attn_dscores: dP = dctx V^T
 * on the MFMA with dS = P (drop'(dP) - dot) / sqrt(d_k) -> dS (pitch lds) and its latest / legacy
 * rel_shift adjoint -> dbd (pitch ldp) in the epilogue.  Layouts as esp_relpos_attn_probs (dctx,
 * ctx (B*T, H*dk) rows of pitch ldd / ldc; V rows at vmat + (b*T + j)*ldv + h*dk; attn / dS
 * (Z,T) rows of pitch lds, 16-B aligned).  Replaces the dP GEMM + esp_attn_softmax_bwd_relpos
 * (attention.py:64-96, 145-165 backward). */
int esp_attn_bwd_prep(const float* dctx, long ldd, const float* ctx, long ldc, int nb, int H, int dk, int T,
                      float* dot, float* dbd, long ldp, int relpos, void* stream);
int esp_attn_dscores(const float* dctx, long ldd, const float* vmat, long ldv, const float* attn, const float* dot,
                     float* dS, float* dbd, long ldp, int relpos, int nb, int H, int dk, float sqrt_dk,
                     float drop_p, unsigned long long seed, int T, long lds, void* stream);
/* Rel-pos attention probabilities for latest (relpos 1: p has P = 2T-1 rows) AND legacy
 * (relpos 2: p has P = T rows, legacy rel_shift attention.py:145-165) rel_shift, one wave per
 * 16 query rows with every score row in registers (no block synchronisation): ac and the bd band
 * on v_mfma_f32_16x16x4_f32, rel_shift through a per-wave LDS ring, key mask, softmax, dropout
 * copy.  Operands as esp_relpos_attn_fwd; d_k = 64, T <= 512; attn / pdrop 16-B aligned with
 * lds % 4 == 0 (columns T .. round_up(T, 4) - 1 of the pitch are written as 0).  Replaces, for these shapes, the
 * reference's matrix_ac / matrix_bd matmuls + rel_shift + softmax + dropout
 * (attention.py:240-263, 64-96). */
/* ABI 31: the relpos_probs_lds_kernel LDS slot-schedule check (attention.hip; a debug build, make
 * VARIANT=_slotchk EXTRA=-DESP_ATTN_SLOT_CHECK=1): slot-generation mismatches counted since the last call
 * (the count is reset), -1 in a build without the check. */
int esp_attn_slot_check_errors(void);
int esp_relpos_attn_probs(const float* qu, const float* qv, const float* kmat, long ldk, const float* p,
                          long ldp_row, int relpos, int nb, int H, float sqrt_dk, const int* klen,
                          float* attn, float* pdrop, float drop_p, unsigned long long seed, int T,
                          long lds, const int* tvalid, void* stream);
/* tvalid (esp_relpos_attn_probs, esp_attn_softmax_bwd_relpos; legacy only, may be NULL): device int
 * T' <= T when the batch is a length bucket padded from T' to T frames.  The legacy rel_shift then
 * uses the reference batch's table positions j + T'-1-i (they depend on T'; the latest ones, i - j,
 * do not), and the adjoint writes the unpadded dbd zero-extended (rows and columns >= T' are 0). */

/* ---- feature front end: DefaultFrontend + GlobalMVN
 * esp_fbank_fwd: STFT (center, reflect, window of length n_fft, onesided) -> power -> mel
 * (dense (n_fft/2+1, n_mels) matrix, band [mel_lo[m], mel_hi[m]) nonzero) -> clamp 1e-10 ->
 * log; frames t >= lens[b]/hop + 1 written as 0 (default.py:82-131, stft.py:63-160,
 * log_mel.py:57-81).  wave (B, N) row pitch ldw; lens (device int32, samples); twiddle
 * n_fft (cos, -sin) pairs of exp(-2 pi i j / n_fft); out (B, T, n_mels), T = N/hop + 1.
 * n_fft even in [16, 2048]: radix-2 FFT when a power of two, direct DFT otherwise.
 * nvalid (may be NULL): device int N' <= N, the reference batch's sample count when the batch is
 * padded to a length bucket: the centre padding reflects at N' (frames >= N'/hop + 1 are 0). */
int esp_fbank_fwd(const float* wave, long ldw, const int* lens, int B, int N, int n_fft, int hop,
                  const float* window, const float* twiddle, const float* melw, const int* mel_lo,
                  const int* mel_hi, int n_mels, float* out, int T, const int* nvalid, void* stream);
/* GlobalMVN in place: x (B,T,F) -> ((x - mean), frames t >= lens[b] zeroed) / std
 * (global_mvn.py:67-90). */
int esp_global_mvn(float* x, const int* lens, int B, int T, int F, const float* mean,
                   const float* stdv, int norm_means, int norm_vars, void* stream);

/* ---- Conv2dSubsampling (subsampling.py:53-87), NHWC */
int esp_conv1_fwd(const float* x, const float* W, const float* bias, float* z, int B, int T,
                  int F, int D, void* stream);
/* esp_conv1_fwd writing z's bf16 copy (RNE) to z16 too (8-B aligned): the bf16 mode's conv2 operand. */
int esp_conv1_fwd_bf16(const float* x, const float* W, const float* bias, float* z, void* z16, int B, int T, int F,
                       int D, void* stream);
/* ABI 32: esp_conv1_fwd (z16 optional, as esp_conv1_fwd_bf16) also writing the ReLU mask as a packed bit map:
 * bit c % 32 of zbits[p * D/32 + c / 32] = (z[p][c] > 0), D % 32 == 0, 4-B aligned (replaces the fp32 map
 * as the conv2 input gradient's mask operand: esp_conv2_dgrad_bits reads 1/32 of the bytes). */
int esp_conv1_fwd_bits(const float* x, const float* W, const float* bias, float* z, void* z16, unsigned* zbits, int B,
                       int T, int F, int D, void* stream);
/* conv2 input gradient as 4 implicit GEMMs (one per parity class of the conv1 output grid):
 * dz1 = relu'(z1) * conv_transpose(dz2, W), W = Conv2d(D,D,3,2).weight (o,c,kt,kf) as the
 * reference stores it; no 9x column buffer.  zeros16: >= 16 B of zeros (device); wc_work:
 * 9*D*D floats (the per-class weight re-layout).  D % 32 == 0. */
int esp_conv2_dgrad(const float* dz2, const float* W, const float* z1, float* dz1, int B, int T1, int F1,
                    int D, const float* zeros16, float* wc_work, long work_bytes, void* stream);
/* ABI 32: esp_conv2_dgrad / esp_conv2_dgrad_bf16 with the conv1 ReLU mask from esp_conv1_fwd_bits' bit map
 * (z1bits) instead of the fp32 map; exactly one of dz2 (fp32) / dz2_16 (bf16, D % 64 == 0) non-NULL. */
int esp_conv2_dgrad_bits(const float* dz2, const void* dz2_16, const float* W, const unsigned* z1bits, float* dz1,
                         int B, int T1, int F1, int D, const float* zeros16, float* wc_work, long work_bytes,
                         void* stream);
/* ABI 32: esp_conv2_dgrad_bits with conv1's weight / bias gradient folded into the class GEMMs' epilogue
 * (replaces esp_conv2_dgrad_bits + esp_conv1_wgrad, subsampling.py:53-87 backward): dW (D x 9) += sum over the
 * conv1 map of dz1 * x-patch, db (D) += sum of dz1, dz1 never materialised.  x: the conv1 input (B, T, F) as
 * esp_conv1_fwd took it; c1_work: esp_conv2_c1fold_workspace_bytes() (per-block partial records + their
 * fixed-order reduction: deterministic).  D % 128 == 0, D <= 512. */
int esp_conv2_dgrad_c1fold(const float* dz2, const void* dz2_16, const float* W, const unsigned* z1bits,
                           const float* x, int T, int F, float* dW, float* db, int B, int T1, int F1, int D,
                           const float* zeros16, float* wc_work, long work_bytes, float* c1_work,
                           long c1_work_bytes, void* stream);
long esp_conv2_c1fold_workspace_bytes(void);
int esp_col2im_relu(const float* dcol, const float* z1, float* dz1, int B, int T1, int F1, int D,
                    void* stream);
int esp_conv1_wgrad(const float* x, const float* dz1, float* dW, float* db, int B, int T, int F,
                    int D, float* work, long work_bytes, void* stream);
/* ABI 31: input_layer "conv2d6" (espnet/nets/pytorch_backend/transformer/subsampling.py:101-146
 * Conv2dSubsampling6: its second Conv2d(D, D, 5, 3)) on explicit columns.  NHWC x [B, T1, F1, C] ->
 * col [B*T2*F2, k*k*C] with row p = (b, t2, f2), column (kt*k + kf)*C + c, T2 = (T1-k)/s + 1,
 * F2 = (F1-k)/s + 1 (a KC x KC GEMM with the (o, kt, kf, c) weight is then the convolution);
 * col2im_relu_nhwc: dx = relu'(z) * the column adjoint (taps summed kt, kf ascending).  C % 4 == 0. */
int esp_im2col_nhwc(const float* x, float* col, int B, int T1, int F1, int C, int k, int s, void* stream);
int esp_col2im_relu_nhwc(const float* dcol, const float* z, float* dx, int B, int T1, int F1, int C, int k,
                         int s, void* stream);
int esp_permute3(const float* in, float* out, int O, int Bd, int Ad, int accumulate, void* stream);

/* ---- losses (ctc.py:39-97, label_smoothing_loss.py:41-63, nets_utils.py:299-320,
 *      espnet/nets/pytorch_backend/ctc.py:185-249) */
int esp_log_softmax(const float* x, float* y, long rows, int V, void* stream);
/* Loss internals run in fp64 where fp32 rounding would exceed the 1e-4 loss gate: the CTC
 * alpha/beta recursions (values ~ -10^3), per-utterance nll, per-row label-smoothing KL and
 * the final reductions.  nll (B) and row_loss (R) are fp64; work >= 2*B*T*(2*Umax+1) doubles. */
int esp_ctc_loss(const float* lp, const long long* labels, int Umax, const int* ilen,
                 const int* tlen, int B, int T, int V, int blank, float gscale, int zero_infinity,
                 double* nll, float* grad, double* work, long work_bytes, void* stream);
int esp_label_smoothing(const float* x, const long long* target, long rows, int V, int ignore,
                        float smoothing, float gscale, float* grad, double* row_loss, int* row_stat,
                        void* stream);
/* out4 = {loss_ctc, loss_att, acc, loss}; denom <= 0 selects the length-normalised
 * attention loss (denominator = non-ignored targets, counted on device) and then also
 * writes out4[4] = 1 / that count (out4 must hold 5 floats). */
int esp_reduce_losses(const double* nll, int B, int zero_inf, const double* row_loss,
                      const int* row_stat, int R, float denom, float ctc_w, float* out4,
                      void* stream);
int esp_argmax(const float* x, long long* out, long rows, int V, void* stream);
int esp_ctc_forced_align(const float* lpz, int T, int V, const long long* y, int U, int blank,
                         int* path, long long* out, void* stream);
/* ABI 31: forced_align over a batch (replaces a loop of espnet/nets/pytorch_backend/ctc.py:185-249
 * CTC.forced_align calls, one per utterance): lpz (B, T, V) fp32 log-probs, utterance b uses its first
 * tlen[b] frames and the first ulen[b] labels of row b of y (B, Umax) int64 (tlen / ulen: device int32);
 * out (B, T) int64 labels, -1 past tlen[b] (and for an utterance with no frames or labels);
 * path: B * T * (2 Umax + 1) int32 workspace.  Each row equals esp_ctc_forced_align on that utterance. */
int esp_ctc_forced_align_batch(const float* lpz, int B, int T, int V, const int* tlen, const long long* y,
                               int Umax, const int* ulen, int blank, int* path, long long* out, void* stream);

/* ---- beam-search CTC prefix scoring (espnet/nets/ctc_prefix_score.py:279-359 CTCPrefixScore,
 *      espnet/nets/scorers/ctc.py CTCPrefixScorer; inference)
 * lp: one utterance's (T, V) CTC log-softmax.  States are (T, 2) fp32 rows (log r^n, log r^b).
 * init: r0 = initial state of the <sos> prefix.  score: for NH hypotheses (states r_prev
 * (NH, T, 2), last label last[NH], common output length out_len = len(prefix) - 1) and C
 * candidate labels each (cands (NH, C)), writes r_new (NH, C, T, 2) and log_psi (NH, C);
 * log_psi = log r^n+r^b at T-1 for c == eos, -1e10 for c == blank. */
int esp_ctc_prefix_init(const float* lp, int T, int V, int blank, float* r0, void* stream);
int esp_ctc_prefix_score(const float* lp, int T, int V, const float* r_prev, const long long* last,
                         int out_len, const long long* cands, int NH, int C, int blank, int eos,
                         float* r_new, float* log_psi, void* stream);

/* ---- workspace sizes.  Every launcher that takes a scratch `work` buffer also takes its size
 * in bytes and fails (status -1, esp_last_error) when it is smaller than the size below, which is
 * computed by the same code that picks the launcher's chunking: callers size their buffers from
 * these queries, never from a restated formula.  Pure host arithmetic (no device call). */
long esp_grad_norm_workspace_bytes(long n);
long esp_layernorm_bwd_workspace_bytes(int M, int D);
long esp_colsum_workspace_bytes(int M, int N);
long esp_dwconv1d_wgrad_workspace_bytes(int Bn, int T, int D, int K);
long esp_bn_swish_fwd_workspace_bytes(int M, int D);
long esp_bn_swish_bwd_workspace_bytes(int M, int D);
long esp_conv1_wgrad_workspace_bytes(int B, int T, int F, int D);
long esp_conv2_dgrad_workspace_bytes(int D);
long esp_ctc_loss_workspace_bytes(int B, int T, int Umax);
/* esp_relpos_dp adapts its grouping to the buffer it gets; this is its preferred size */
long esp_relpos_dp_workspace_bytes(int nb, int H, int T);

#ifdef __cplusplus
}
#endif
#endif
