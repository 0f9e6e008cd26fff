/*
 * gnk.h -- C-ABI of libgnk.so, the MI355X (gfx950) hot path of the
 * generalized-Krylov Gauss-Newton solver on the Bratu problem.
 *
 * Reference (mariusbaehr/gauss_newton_via_generalized_krylov_subspaces, read-only
 * at /root/reference in the build container) is pure Python/NumPy/SciPy; there
 * is no native interface to replace.  Each entry point below names the Python
 * expression of the reference it executes on the GPU, so a maintainer can bind
 * it with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer (hipMalloc / torch CUDA tensor)
 *    unless its name ends in _host.  Sizes are element counts.
 *  - All work is enqueued on the stream given to gnk_set_stream (default: the
 *    null stream).  Functions do not synchronise and never allocate (the
 *    context owns a fixed scratch arena made at gnk_ctx_create).
 *  - Return value: 0 = OK, < 0 = error; gnk_last_error(ctx) has the text.
 *  - Grid vectors are "slab vectors": the rank owns global rows
 *    [row0, row0 + nrows) of the N x N interior grid (flat index jx*N + iy, jx
 *    slow, ref:bratu_pde_problem.py:69-74) and stores them with GNK_GHOST_ROWS
 *    ghost rows on each side: length (nrows + 2*GNK_GHOST_ROWS) * N, owned data
 *    at offset GNK_GHOST_ROWS * N.  Ghost rows outside the domain are zero.
 *  - Reductions write their result into a small device array (the caller
 *    combines ranks in rank order); they are deterministic run to run.
 */
#ifndef GNK_H
#define GNK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNK_GHOST_ROWS 2
#define GNK_ABI_VERSION 6

typedef struct gnk_ctx gnk_ctx;

/* ---- context ---------------------------------------------------------- */
int gnk_abi_version(void);
int gnk_ctx_create(int device, gnk_ctx** out);
void gnk_ctx_destroy(gnk_ctx* ctx);
const char* gnk_last_error(const gnk_ctx* ctx);
int gnk_set_stream(gnk_ctx* ctx, void* hip_stream);
/* Compensated (Dot2) reductions -- the CG scalars of gnk_cg_normal_matvec / gnk_cg_step_matvec /
 * gnk_cg_update_xr and sum x**2 of gnk_vec_stats -- are normally returned as one
 * double s + c.  With on != 0 they are returned as the unevaluated pair: out[2j] = s_j,
 * out[2j+1] = c_j (gnk_vec_stats: {s, c, max|x|}), so a multi-rank caller can merge every rank's
 * pair with TwoSum in rank order before rounding (slab.Comm.sum_pairs).  Default 0. */
int gnk_set_reduce_pairs(gnk_ctx* ctx, int on);
/* Rank-count-independent reductions.  seg_rows > 0 splits the grid into fixed global row segments
 * of seg_rows rows (call after gnk_set_bratu; the slab must hold whole segments: row0 % seg_rows ==
 * nrows % seg_rows == 0; at most 64 per slab; gnk_set_bratu resets it to 0).  Every reduction of the
 * GNK path -- the Gram passes of gnk_gram at k <= 20 (N % 128 == 0), the first-trial / pending-column
 * sums (gnk_basis_gemv_vjp_gemv_t*, gnk_basis_gemv_pending), gnk_bratu_residual, gnk_vec_stats,
 * gnk_cgs_update, gnk_vjp_gemv_t, gnk_normalize_jnorm -- is then computed per segment with a block
 * decomposition that depends on N and seg_rows only (every grid that carries partial sums is a fixed
 * function of the geometry and the kernel instance -- never of occupancy or the CU count: gnk_decomp_check),
 * and the segment values are folded pairwise in
 * a fixed tree: v[i] += v[i + w] for w = 1, 2, 4, ... (i a multiple of 2w, i + w < n).  With
 * seg_rows = N / P and P / w segments per rank, combining the w ranks' values in the same tree
 * order (slab.Comm) gives the same bits for every w dividing P.  Compensated pairs
 * (gnk_set_reduce_pairs) stay per rank.  0 = off (the default: one decomposition per slab). */
int gnk_set_segments(gnk_ctx* ctx, int64_t seg_rows);
/* Reductions run on the per-slab decomposition although segments were on, since the context was created:
 * the wide Gram passes (k > 20, or N % 128 != 0) and a Gram grid the segment rows cannot tile.  Those
 * results are rank-count dependent (rounding only); 0 means every reduction so far was segmented.
 * -1 for a NULL context.  Replaces nothing in the reference (multi-rank bookkeeping). */
int64_t gnk_segment_fallbacks(const gnk_ctx* ctx);
/* Kernel-choice overrides for tests and A/B tooling (value 0 = the library's own choice, the
 * default; the solver never sets them):
 *   GNK_TUNE_GRAM_PATH   1 = the staged MFMA Gram kernel for every pass it covers (k <= 20),
 *                        2 = never the staged kernel, 3 = no all-VALU Gram kernels
 *   GNK_TUNE_GRAM_RING   4 / 5 = LDS ring slots of the staged Gram kernel
 *   GNK_TUNE_GRAM_V1MIN  first k of the one-point VALU Gram kernel (-1: never)
 *   GNK_TUNE_CG_MATVEC   1 = the point-wise normal matvec instead of the row-marching one
 *   GNK_TUNE_VJPG_BLOCKS cap on the blocks of gnk_vjp_gemv_t
 *   GNK_TUNE_GRAM_WIDE   1 = never the prefetching wide Gram kernel, 2 = also for 2..3 column blocks,
 *                        3 = the pair-split kernel instead of the VGPR-RinvAug one for 5..7 blocks,
 *                        4 = the VGPR-RinvAug (marching) kernel from 2 column blocks (default: from 3),
 *                        5 = from 5 blocks (3 / 4 blocks on the chunked / prefetching kernels, the round-4 choice)
 *   GNK_TUNE_GRAM_RPR    > 0: grid rows per row range of the staged / VALU Gram kernels (a finer,
 *                        fixed decomposition; A/B of what rank-count-independent partials cost)
 *   GNK_TUNE_LLS         1 = the device least-squares solve on one wave, a column per lane (k_lls), instead of
 *                        one entry per thread on 32 x 32 threads (k_lls_2d); the same bits
 *   GNK_TUNE_VJPG_ZMAX   > 0: at most this many column chunks per gnk_vjp_gemv_t launch (tests: the split
 *                        that wide bases with segments need; the same bits)
 *   GNK_TUNE_DECOMP_LDS  > 0: bytes of extra dynamic LDS per workgroup of the persistent kernels (first trial,
 *                        pending column, marching Gram, CG normal matvec): fewer resident workgroups, the same
 *                        grid -- tests that no result depends on occupancy (the same bits)
 *   GNK_TUNE_TRIALW      16 * depth + workgroups per CU of the wide fused first trial (tooling A/B; the grid is
 *                        its reduction decomposition, so a different per-CU count changes h's last bits)
 *   GNK_TUNE_GRAM_TM     staged Gram, k = 17..20: 1 = the lead columns' sums on VALU for every tail, 2 = on 4x4x4
 *                        f64 MFMA blocks for every tail (tooling A/B and tests; a different summation order)
 *   GNK_TUNE_GRAM_Q      staged Gram: 1 = never the 4x4x4-block form (k_gram_q; k = 8, 9 then on the VALU kernel), 2 = from
 *                        k = 5 (default: k >= 8) */
#define GNK_TUNE_GRAM_PATH 0
#define GNK_TUNE_GRAM_RING 1
#define GNK_TUNE_GRAM_V1MIN 2
#define GNK_TUNE_CG_MATVEC 3
#define GNK_TUNE_VJPG_BLOCKS 4
#define GNK_TUNE_GRAM_WIDE 5
#define GNK_TUNE_GRAM_RPR 6
#define GNK_TUNE_LLS 7
#define GNK_TUNE_VJPG_ZMAX 8
#define GNK_TUNE_DECOMP_LDS 9
#define GNK_TUNE_TRIALW 10
#define GNK_TUNE_GRAM_TM 11
#define GNK_TUNE_GRAM_Q 12
#define GNK_TUNE_COUNT 13
int gnk_set_tuning(gnk_ctx* ctx, int key, int value);
/* doubles in the context's scratch arena (bounds the wide generic Gram: kp * m <= this) */
int64_t gnk_scratch_doubles(void);

/* Bratu slab geometry + coefficients.  h = grid_resolution, alpha = ALPHA,
 * lambda = LAMBDA of BratuPdeProblem (ref:bratu_pde_problem.py:20-67). */
int gnk_set_bratu(gnk_ctx* ctx, int64_t N, int64_t row0, int64_t nrows,
                  double h, double alpha, double lambda);
int64_t gnk_slab_len(const gnk_ctx* ctx);

/* ---- Bratu operator (matrix-free; replaces the per-call CSR assembly) --- */
/* out = J(u) @ v on owned rows; v's ghost rows must be valid.
 * J(u) = -(L + ALPHA*D_x + LAMBDA*diag(exp u))      ref:bratu_pde_problem.py:88-96 */
int gnk_bratu_jvp(gnk_ctx* ctx, const double* u, const double* v, double* out);
/* out = J(u).T @ w on owned rows               ref:krylow.py:62 (jac_ev.T @ res_ev) */
int gnk_bratu_vjp(gnk_ctx* ctx, const double* u, const double* w, double* out);
/* F = pde_operator(x) on owned rows             ref:bratu_pde_problem.py:76-83 */
int gnk_bratu_forward(gnk_ctx* ctx, const double* x, double* F);
/* r = y - pde_operator(x) on owned rows and the one ghost row each side that
 * lies inside the domain (x must be valid on owned +-2 rows);
 * norm2_out[0] = sum(r**2) over owned rows      ref:bratu_pde_problem.py:85-86,
 *                                               ref:armijo_goldstein.py:49,57 */
int gnk_bratu_residual(gnk_ctx* ctx, const double* x, const double* y, double* r,
                       double* norm2_out);
/* out = diag(J(u).T @ J(u)) (closed form), or 1 / that when reciprocal != 0
 * (the Jacobi preconditioner)                   ref:gauss_newton.py:50-54 */
int gnk_bratu_diag_jtj(gnk_ctx* ctx, const double* u, double* out, int reciprocal);
/* d = diagonal of L + ALPHA*D_x + LAMBDA*diag(exp u) on owned +-1 rows (inside
 * the domain); u must be valid there        ref:bratu_pde_problem.py:92-96 */
int gnk_bratu_jdiag(gnk_ctx* ctx, const double* u, double* d);

/* ---- generalized Krylov basis (column-major V, column stride ldv) -------- */
/* x = V[:, :k] @ c over the whole slab (ghost rows included)
 *                                               ref:krylow.py:41-42 */
int gnk_basis_gemv(gnk_ctx* ctx, const double* V, int64_t ldv, int k,
                   const double* c, double* x);
/* g = -(J(u).T @ r) on owned rows, h = V[:, :k].T @ g (local partial; k may
 * be 0, then only g is written and h_out may be NULL)
 *                                               ref:krylow.py:62,64 */
int gnk_vjp_gemv_t(gnk_ctx* ctx, const double* u, const double* r,
                   const double* V, int64_t ldv, int k, double* g, double* h_out);
/* Fused first Armijo trial + basis-update products (version "res_old"): x = V[:, :k] @ c on
 * the whole slab (rounding of gnk_basis_gemv), then on owned rows g = -(J(x)^T r) and
 * h = V[:, :k]^T g -- gnk_basis_gemv followed by gnk_vjp_gemv_t(u = x) from one read of V.
 * 1 <= k <= 24 (a point's basis row in VGPRs); 25 <= k <= 208 when N % 128 == 0, ldv is even and
 * segments are off (tiles of V through LDS; x and w then sum the columns in four blocked quarters,
 * not in one sequence).   ref:krylow.py:42, :62, :64 + gauss_newton_krylow.py:91,115 */
int gnk_basis_gemv_vjp_gemv_t(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, const double* r,
                              double* x, double* g, double* h_out);

/* Deferred Gram-Schmidt: the basis update of ref:krylow.py:62-73 stores the raw
 * g = -J^T r as column k of V ("pending") and its projection coefficients hh; the next least-
 * squares pass sees J w through its triangular transform, and the first Armijo trial point
 * materialises w = g - V[:, :k] @ hh in place over column k (whole slab, the rounding of
 * gnk_cgs_update) while it reads V anyway:
 *   x = V[:, :k] @ c[:k] + w c[k]   (rounding of gnk_basis_gemv over k + 1 columns),
 *   stats_out = {sum w**2, max|w|} over owned rows (the norm and breakdown test, ref:krylow.py:66,71).
 * x must not alias column k.                      ref:krylow.py:41-42, 64-71 */
int gnk_basis_gemv_pending(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, const double* hh,
                           double* x, double* stats_out);
/* gnk_basis_gemv_vjp_gemv_t with the pending column k materialised as in gnk_basis_gemv_pending:
 * x and h_out cover k + 1 columns (h_out[k] = w . g), stats_out as above.  1 <= k + 1 <= 24, or up to
 * 208 as gnk_basis_gemv_vjp_gemv_t; g must not alias column k.        ref:krylow.py:42, :62-71 + gauss_newton_krylow.py:91,115 */
int gnk_basis_gemv_vjp_gemv_t_pending(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c,
                                      const double* hh, const double* r, double* x, double* g, double* h_out,
                                      double* stats_out);

/* One preconditioned CholeskyQR least-squares solve on the device (lls.py), from a
 * Gram G (kp x kp, row-major, already summed over ranks) of [J V T | r]: optionally rescale the last
 * column (P[k-1][k-1] = sqrt(G[k-1][k-1])), G[:k,:k] = Ry^T Ry, z = Ry^-T G[:k,k], R = Ry P,
 * d = -R^-1 z, jdd = ||R d||^2, e_try = e + sdd * d (elementwise).  P: k x k upper triangular.
 * out = [status (0 ok, 1 not SPD), jdd, s, d (k), R (k*k), Ry (k*k), R^-1 (k*k)].
 * 1 <= k <= gnk_lls_max_k().           ref:gauss_newton_krylow.py:16-36, armijo_goldstein.py:50 */
/* out[j] = sum over p of parts[p * n + j] in the fixed pairwise order of gnk_set_segments' fold
 * (v[i] += v[i + w] for w = 1, 2, 4, ..; the order slab.Comm sums all-gathered partials on the host):
 * the cross-rank reduction of a small per-rank vector after all_gather. */
int gnk_rank_sum(gnk_ctx* ctx, const double* parts, int world, int64_t n, double* out);
int gnk_lls_max_k(void);
int gnk_lls_solve(gnk_ctx* ctx, const double* G, int kp, int k, const double* P, int rescale, const double* sdd,
                  const double* e, double* out, double* e_try);
/* The next step's least-squares inputs on the device, assuming this step (k columns, the last one
 * pending if pending != 0) accepts its first trial and appends a pending column with the rank-summed
 * raw products h = pack[3:3+k] (pack[1] = sum w**2 of this step's pending column): sc_next, hh_next
 * (k), the augmented transform T_next (kp_next x kp_next) = [[diag(sc') D R^-1, -hh'], [0, 1]] (+ r),
 * P_next = blockdiag(R_true, 1) ((k+1) x (k+1)), sdd_next = [sc', 1], e_next = [e_try, 0].
 * Lets the host enqueue step i+1 before it has read step i.
 *                                         ref:krylow.py:64-73, gauss_newton_krylow.py:98,124 */
int gnk_lls_next(gnk_ctx* ctx, int k, int pending, const double* out, const double* e_try, const double* pack,
                 const double* sc, int kp_next, double* T_next, double* P_next, double* sdd_next, double* e_next,
                 double* hh_next, double* sc_next);

/* g -= V[:, :k] @ h on owned rows; stats_out = {sum g**2, max|g|}
 *                                               ref:krylow.py:64,66,71 */
int gnk_cgs_update(gnk_ctx* ctx, const double* V, int64_t ldv, int k,
                   const double* h, double* g, double* stats_out);
/* stats_out = {sum x**2, max|x|} over owned rows  ref:krylow.py:31,36 */
int gnk_vec_stats(gnk_ctx* ctx, const double* x, double* stats_out);
/* dst = src / denom on owned rows (full_slab = 0) or the whole slab (1)
 *                                               ref:krylow.py:37,71 */
int gnk_vec_div(gnk_ctx* ctx, const double* src, double denom, double* dst, int full_slab);

/* v = g / denom on the whole slab (g's ghost rows must already hold the
 * neighbours' rows) and *jnorm2_out = sum over owned rows of (J(u) g)^2 in one
 * pass: the new basis column of ref:krylow.py:71 plus ||J v_new||^2 * denom^2,
 * the column scale of the next least-squares preconditioner.
 * v != g. */
int gnk_normalize_jnorm(gnk_ctx* ctx, const double* u, const double* g, double denom, double* v,
                        double* jnorm2_out);

/* out = x + (alpha * d) (two roundings, as NumPy's x + t * d) on owned rows or
 * the whole slab                                ref:gauss_newton.py:125,
 *                                               ref:armijo_goldstein.py:56 */
int gnk_vec_axpy(gnk_ctx* ctx, const double* x, double alpha, const double* d, double* out,
                 int full_slab);

/* ---- Gram passes of the CholeskyQR2 least-squares solve (fp64 MFMA) ----
 * W = [J(u) @ V[:, :k] | r] @ RinvAug  (RinvAug: kp x kp row-major, ld = kp: the
 * inverse of the pass-1 R factor, 1 at [k][k] when r is given, zeros elsewhere;
 * NULL = identity; r: NULL = no extra column).
 * G_out (kp x kp, kp = k (+1 if r) rounded up to 16, row-major) = W.T @ W
 * over owned rows.  This replaces scipy.linalg.qr(-J@V) + q.T @ y of
 *                                               ref:gauss_newton_krylow.py:30,35 */
int gnk_gram_padded_dim(int k, int with_r);
int gnk_gram(gnk_ctx* ctx, const double* u, const double* V, int64_t ldv, int k,
             const double* rinv, int64_t ldr, const double* r, double* G_out);

/* ---- CGLS (scipy cg on A.T A, A = -J)     ref:gauss_newton.py:11-60 ----- */
/* q = A.T @ (A @ p) = J.T (J p), A = -J, as one fused 13-point stencil over the
 * precomputed diagonal d (gnk_bratu_jdiag); p valid on owned +-2 rows.
 * pq_out[0] = p . q over owned rows        ref:gauss_newton.py:36, scipy iterative.py:411-412 */
int gnk_cg_normal_matvec(gnk_ctx* ctx, const double* d, const double* p, double* q,
                         double* pq_out);
/* One CG iteration's direction update + normal matvec in one pass (N even):
 * p_out = z (first) or p_in * beta + z on owned and slab ghost rows (z's ghost rows
 * exchanged), q = J.T (J p_out), pq_out[0] = p_out . q (owned); if x != NULL also
 * x += xalpha * p_in on owned rows (the previous iteration's update, applied one
 * iteration late).  p_out must not alias p_in.   scipy iterative.py:401-415 */
int gnk_cg_step_matvec(gnk_ctx* ctx, const double* d, const double* z, const double* p_in,
                       double* p_out, double* q, double beta, int first, double* x,
                       double xalpha, double* pq_out);
/* x += alpha p (skipped when x is NULL) ; r -= alpha q ; z = dinv * r (or r if dinv NULL);
 * out = {r . r, r . z} (owned)              scipy iterative.py:401-415 */
int gnk_cg_update_xr(gnk_ctx* ctx, double alpha, const double* p, const double* q,
                     double* x, double* r, const double* dinv, double* z, double* out);
/* The same two kernels with their coefficients read from a device CG state (8 doubles, written by
 * gnk_cg_scalars): beta = state[0], the lagged x update's alpha = state[1] (step matvec), alpha =
 * state[2] (update).  No host value between the kernels of an iteration; the same bits as the host-
 * coefficient forms given the same values.          scipy iterative.py:401-415 */
int gnk_cg_step_matvec_dev(gnk_ctx* ctx, const double* d, const double* z, const double* p_in,
                           double* p_out, double* q, int first, double* x, const double* state,
                           double* pq_out);
int gnk_cg_update_xr_dev(gnk_ctx* ctx, const double* state, const double* p, const double* q,
                         double* x, double* r, const double* dinv, double* z, double* out);
/* The scalar recurrence of the fused iteration on the device.  parts: world ranks' compensated pairs
 * (gnk_set_reduce_pairs on), merged in rank order exactly as slab.Comm.merge_pairs (TwoSum; one
 * rank: s + c).  stage 0: parts = rank x {r.r, r.z} of the alpha = 0 update -> state[5] = r.r,
 * state[3] = rho = r.z; stage 1: parts = rank x {p.q} -> state[6] = p.q, state[2] = rho / p.q;
 * stage 2: parts = rank x {r.r, r.z} -> state[5] = r.r, state[4] = rho, state[3] = r.z,
 * state[0] = state[3] / state[4], state[1] = state[2].  One launch of one thread.
 * Replaces the host's alpha = rho / p.q, beta = rho / rho_prev (scipy iterative.py:401-415) and the
 * host merge of per-rank pairs (the two host reads per CG iteration of ref:gauss_newton.py:36-58). */
int gnk_cg_scalars(gnk_ctx* ctx, const double* parts, int world, int stage, double* state);
/* p = z (first) or p = beta * p + z (owned rows) */
int gnk_cg_update_p(gnk_ctx* ctx, double beta, int first, const double* z, double* p);
/* Single-reduction CG (Chronopoulos-Gear) iteration update, the non-parity option of gauss_newton
 * (cg_variant="single_reduction"), owned rows: p = u + beta p, s = w + beta s (first != 0:
 * p = u, s = w); x += alpha p; r -= alpha s; u = dinv * r (dinv NULL: u = r);
 * out[0] = r . u, out[1] = r . r.  w = A^T A u comes from gnk_cg_normal_matvec (its u . w).
 *                                   restates scipy iterative.py:401-415 with one reduction */
int gnk_cg_sr_update(gnk_ctx* ctx, double alpha, double beta, int first, const double* w, double* p, double* s,
                     double* x, double* r, const double* dinv, double* u, double* out);


/* ---- generic problems: flat length-n vectors, no gnk_set_bratu needed ------ */
/* x = V[:, :k] @ c                                                    ref:krylow.py:41-42 */
int gnk_flat_gemv(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, double* x, int64_t n);
/* h = V[:, :k]^T g (deterministic)                                   ref:krylow.py:64 (inner) */
int gnk_flat_gemv_t(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* g, int64_t n, double* h_out);
/* g -= V[:, :k] @ h ; stats_out = {sum g^2, max|g|}            ref:krylow.py:64, :66, :71 */
int gnk_flat_cgs_update(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* h, double* g, int64_t n,
                        double* stats_out);
/* {sum x^2, max |x|}; a . b; dst = src / denom; out = x + (alpha * d) */
int gnk_flat_stats(gnk_ctx* ctx, const double* x, int64_t n, double* stats_out);
int gnk_flat_dot(gnk_ctx* ctx, const double* a, const double* b, int64_t n, double* out);
int gnk_flat_div(gnk_ctx* ctx, const double* src, double denom, double* dst, int64_t n);
int gnk_flat_axpy(gnk_ctx* ctx, const double* x, double alpha, const double* d, double* out, int64_t n);
/* CG vector updates on flat vectors (as gnk_cg_update_xr / gnk_cg_update_p) */
int gnk_flat_cg_update_xr(gnk_ctx* ctx, double alpha, const double* p, const double* q, double* x, double* r,
                          const double* dinv, double* z, int64_t n, double* out);
int gnk_flat_cg_update_p(gnk_ctx* ctx, double beta, int first, const double* z, double* p, int64_t n);
/* y = A x, CSR with 32-bit indices, scipy csr_matvec summation order: the J @ v / J.T @ w of a
 * user Jacobian (J.T as the CSR of the transpose).  mode 1: y = -(A x); mode 2: y = 1 / (A x)
 * (with the squared entries of J.T and x = 1: the Jacobi vector 1 / diag(A.T @ A))
 *                    ref:krylow.py:62, gauss_newton_krylow.py:86, gauss_newton.py:36, :50-52 */
int gnk_csr_spmv(gnk_ctx* ctx, int64_t nrows, const int* indptr, const int* indices, const double* data,
                 const double* x, double* y, int mode);
/* Gram of [W @ RinvAug | r] for a materialised W (k <= 63 columns of length m, stride ldw),
 * G_out kp x kp (kp = gnk_gram_padded_dim(k, r != NULL)); rinv NULL = identity
 *                                                       ref:gauss_newton_krylow.py:16-36, 86-89 */
int gnk_flat_gram(gnk_ctx* ctx, const double* W, int64_t ldw, int k, const double* rinv, int64_t ldr,
                  const double* r, int64_t m, double* G_out);

/* ---- tooling (not on the solver path) ----------------------------------- */
/* Per-launch HIP-event timer for kernel classes (bench roofline): after
 * gnk_timer_start (one class; gnk_timer_add puts more classes in the same
 * window), the next `capacity` launches of those kernels are bracketed by an
 * event pair on the context's stream; gnk_timer_collect(_ids) synchronises them
 * and returns the count, the milliseconds, the algorithmic bytes (and the class)
 * of each launch in launch order. */
#define GNK_TIMER_GRAM 1
#define GNK_TIMER_JVP 2
#define GNK_TIMER_CG_MATVEC 3
#define GNK_TIMER_TRIAL 4   /* first Armijo trial + update products, k_gemv_vjpg */
#define GNK_TIMER_PROBE 5   /* gnk_probe_stream */
#define GNK_TIMER_CG_XR 6   /* CG r -= alpha q, z = M r (+ x += alpha p), k_cg_xr */
#define GNK_TIMER_CG_AUX 7  /* CG reductions of the partials (wreduce2) and k_cg_scalars; 0 bytes */
int gnk_timer_start(gnk_ctx* ctx, int kernel_id, int capacity);
int gnk_timer_add(gnk_ctx* ctx, int kernel_id);
int gnk_timer_collect(gnk_ctx* ctx, double* ms_out, double* bytes_out, int capacity);
int gnk_timer_collect_ids(gnk_ctx* ctx, double* ms_out, double* bytes_out, int* ids_out, int capacity);
/* The persistent reduction kernels' fixed grids (workgroups per CU x 256, a table per kernel instance, see
 * GNK_TUNE_DECOMP_LDS) beside this device's live occupancy (hipOccupancyMaxActiveBlocksPerMultiprocessor) for
 * the same instances: table_out[i] / live_out[i] for i < min(return value, capacity); returns the instance
 * count.  A mismatch costs time (partly filled rounds), never bits. */
int gnk_decomp_check(gnk_ctx* ctx, int* table_out, int* live_out, int capacity);
/* back-to-back v_mfma_f64_16x16x4_f64 issue-rate probe: blocks x 256 threads,
 * 4 independent accumulators per wave, iters x 4 MFMAs per wave */
int gnk_probe_mfma_f64(gnk_ctx* ctx, double* out, int blocks, int iters);
/* HBM streaming floor: mode 0 triad a = b + s c, 1 read-only (sum of b into scratch), 2 copy a = b;
 * n doubles (even), 16-B accesses; timed as GNK_TIMER_PROBE with 24 n / 8 n / 16 n bytes */
int gnk_probe_stream(gnk_ctx* ctx, double* a, const double* b, const double* c, double s, int64_t n, int mode);

#ifdef __cplusplus
}
#endif
#endif /* GNK_H */
