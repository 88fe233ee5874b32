/*
 * quill_gpu.h — C-ABI of the MI355X (gfx950) prover hot path for Quill.
 *
 * Drop-in boundary for gio54321/quill-zkvm (reference mounted at /root/reference):
 * every entry point below names the reference item it replaces (file:line).
 * A Rust shim binds these with `extern "C"` and keeps the
 * reference's `MultilinearPCS` / `SumcheckProof` / `ZeroCheckProof` surfaces.
 *
 * Conventions
 *  - Field elements (BN254 Fr and Fq) are 4 x uint64 little-endian limbs in
 *    Montgomery form with R = 2^256: exactly arkworks' in-memory
 *    `Fp256(BigInt([u64; 4]))`, so a Rust shim passes `&[Fr]` as a pointer
 *    with no conversion.
 *  - A G1 point is `uint64_t xy[8]` (x limbs then y limbs, Montgomery) plus an
 *    infinity flag (`uint8_t`), i.e. ark-ec `Affine<G1Config>` field order.
 *  - The Fiat-Shamir transcript (transcript/src/transcript.rs:5-74) is carried
 *    as its 32-byte BLAKE3 chaining state `uint8_t state[32]`, updated in place.
 *  - Every function returns an int status: 0 = QG_OK, < 0 = error.  Nothing
 *    unwinds across the ABI; qg_last_error() describes the last failure on a
 *    context.  The reference prover panics where these return
 *    QG_ERR_INVALID / QG_ERR_ASSERT (pcs/src/kzg.rs:62-65,85,
 *    hyperplonk/src/piops/multiset_check.rs:51,63); a Rust shim maps a non-zero
 *    status to `panic!` to keep those semantics.
 *  - Calls are synchronous (they may use internal HIP streams).  A context is
 *    bound to one device; use one context per thread.
 */
#ifndef QUILL_GPU_H
#define QUILL_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QG_OK 0
#define QG_ERR_INVALID (-1)     /* bad argument / size (reference: assert! panic) */
#define QG_ERR_DEVICE (-2)      /* HIP runtime error */
#define QG_ERR_OOM (-3)         /* device allocation failed */
#define QG_ERR_UNSUPPORTED (-4) /* expression / size outside the supported envelope */
#define QG_ERR_ASSERT (-5)      /* prover-side sanity check failed (reference: assert!) */
#define QG_ERR_COMM (-6)        /* RCCL failure */

typedef struct qg_ctx qg_ctx;
typedef struct qg_srs qg_srs;
typedef struct qg_buf qg_buf;

/* ---------------------------------------------------------------- context */
/* Device context (one HIP device, its streams and scratch). */
int qg_ctx_create(int device, qg_ctx** out);
int qg_ctx_destroy(qg_ctx* ctx);
const char* qg_last_error(const qg_ctx* ctx);
/* Library / build identification (e.g. "gfx950"). */
const char* qg_version(void);

/* Multi-GPU: attach an RCCL communicator (one process per GPU).  `unique_id`
 * is the 128-byte ncclUniqueId produced by qg_comm_unique_id() on rank 0 and
 * broadcast by the caller (e.g. torch.distributed).  After this, qg_msm_g1 /
 * qg_kzg_commit on an SRS *shard* return the sum over all ranks, and
 * qg_sumcheck_prove treats its tables as the rank's block of the hypercube
 * (high index bits = rank). */
int qg_comm_unique_id(uint8_t out_id[128]);
/* world == 1 detaches (plain single-GPU paths) unless QG_FORCE_RCCL=1 is set:
 * then a real one-rank RCCL communicator is attached (unique_id may be NULL)
 * and the sharded code paths run through it — a test switch so a 1-GPU box
 * executes the RCCL transport. */
int qg_ctx_attach_comm(qg_ctx* ctx, int rank, int world, const uint8_t unique_id[128]);
/* What the context exchanges through: 0 none (single GPU), 1 the in-process
 * loopback, 2 an RCCL communicator.  `sharded` = 1 when the sharded paths run. */
int qg_ctx_comm_info(const qg_ctx* ctx, int* kind, int* rank, int* world, int* sharded);
/* In-process loopback group: `world` contexts, each driven by its own host
 * thread (possibly on one device), exchange through device-to-device copies
 * instead of RCCL.  Exercises every sharded path on a single GPU. */
typedef struct qg_loopback qg_loopback;
int qg_loopback_create(int world, qg_loopback** out);
int qg_loopback_destroy(qg_loopback* lb);
int qg_ctx_attach_loopback(qg_ctx* ctx, qg_loopback* lb, int rank);
/* Allgather of `bytes` host bytes from every rank into recv (world * bytes, rank
 * order) over the attached communicator: the host-side agreement steps of the
 * sharded prover (constraint-check verdicts, boundary rows). */
int qg_comm_allgather_host(qg_ctx* ctx, const void* send, size_t bytes, void* recv);
/* Personalised exchange of host bytes: send holds world chunks of `bytes` (chunk d
 * goes to rank d), recv receives world chunks (chunk s came from rank s); the
 * collective the sharded S polynomial uses (grouped RCCL send/recv). */
int qg_comm_alltoall_host(qg_ctx* ctx, const void* send, size_t bytes, void* recv);
/* The full witness of a trace, concat(columns) (hyperplonk/src/proof/proof.rs:270),
 * as this rank's block: every rank passes its row block (rows / world entries)
 * of each of the `ncols` columns and receives entries
 * [rank * ncols * rows / world, (rank + 1) * ncols * rows / world) of the
 * column-major flattening (exchanged with one RCCL allgather of the packed
 * row blocks, then a local extraction).
 * world == 1: the plain concatenation. */
int qg_trace_full_witness(qg_ctx* ctx, const qg_buf* const* col_blocks, uint32_t ncols,
                          uint64_t rows, qg_buf* full_block);

/* ---------------------------------------------------------------- transcript */
/* Transcript::new(domain)                  transcript/src/transcript.rs:14-22 */
int qg_transcript_new(const uint8_t* domain, size_t len, uint8_t state[32]);
/* Transcript::append_bytes(msg)            transcript.rs:25-31 */
int qg_transcript_append(uint8_t state[32], const uint8_t* msg, size_t len);
/* Transcript::draw_challenge(n) (n <= 64)  transcript.rs:48-62 */
int qg_transcript_draw(uint8_t state[32], uint8_t* out, size_t n);
/* Transcript::draw_field_element::<Fr>()   transcript.rs:70-74 (out: Montgomery) */
int qg_transcript_draw_fr(uint8_t state[32], uint64_t out_fr[4]);
/* ark-serialize uncompressed encodings used with append_serializable
 * (transcript.rs:33-37): Fr -> 32 B canonical LE; G1 -> 64 B (x||y, SW flags). */
int qg_fr_serialize(const uint64_t fr[4], uint8_t out[32]);
int qg_g1_serialize(const uint64_t xy[8], uint8_t infinity, uint8_t out[64]);

/* ---------------------------------------------------------------- SRS */
/* Upload `n` affine bases (KZG::g1_points, pcs/src/kzg.rs:10-23), x||y Montgomery
 * limbs per point (n x 8 uint64) + per-point infinity flags (may be NULL).
 * The device keeps the bases affine (this removes the per-commit
 * `into_affine` of every SRS point, kzg.rs:67-71) together with the MSM's
 * precomputed window-shifted copies. */
int qg_srs_upload(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                  qg_srs** out);
/* Bases for one-shot MSMs (VariableBaseMSM::msm_unchecked over bases used
 * once, the call at pcs/src/kzg.rs:72 with a base slice that is not a fixed
 * SRS): same layout and MSM results as qg_srs_upload, but only ONE table is
 * built (no window-shifted copies: 1/W of the HBM and none of the W - 1 shift
 * passes, 0.63 s at 2^24).  Every MSM over these bases then bins its W windows
 * in W passes and combines the window sums by Horner steps; use qg_srs_upload
 * for bases that serve many MSMs.  Any qg_* call taking a qg_srs accepts it. */
int qg_bases_upload(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                    qg_srs** out);
/* KZG::trusted_setup with an explicit tau (kzg.rs:35-59): bases [tau^i] g for
 * i < n, generated on the device.  `g_xy` NULL = the BN254 generator (1, 2). */
int qg_srs_generate(qg_ctx* ctx, const uint64_t tau[4], const uint64_t* g_xy, size_t n,
                    qg_srs** out);
/* Bases [tau^(offset+i)] g for i < n: the shard [offset, offset+n) of a larger
 * SRS (one shard per rank for the multi-GPU MSM). */
int qg_srs_generate_range(qg_ctx* ctx, const uint64_t tau[4], const uint64_t* g_xy,
                          uint64_t offset, size_t n, qg_srs** out);
int qg_srs_destroy(qg_srs* srs);
size_t qg_srs_len(const qg_srs* srs);
/* MSM window geometry of this SRS: signed-digit window bits c and window
 * count W (the tables hold W shifted copies of the bases; one table for
 * qg_bases_upload). */
int qg_srs_window_info(const qg_srs* srs, int* c, int* windows);
/* Copy bases [offset, offset+n) back to the host (affine, Montgomery). */
int qg_srs_download(const qg_srs* srs, size_t offset, size_t n, uint64_t* affine_xy,
                    uint8_t* infinity);

/* ---------------------------------------------------------------- device vectors */
/* Fr vectors resident in HBM (for callers that keep witnesses on the device). */
int qg_buf_create(qg_ctx* ctx, size_t n, qg_buf** out);
int qg_buf_destroy(qg_buf* buf);
size_t qg_buf_len(const qg_buf* buf);
int qg_buf_upload(qg_buf* buf, const uint64_t* fr, size_t n);
int qg_buf_download(const qg_buf* buf, uint64_t* fr, size_t n);
/* Fill with uniform Fr from splitmix64->xoshiro256** keyed by (seed, index
 * block); used for synthetic benchmark witnesses. */
int qg_buf_fill_random(qg_buf* buf, uint64_t seed);
/* Non-owning view of entries [offset, offset+n) of `base` (destroy it with
 * qg_buf_destroy; the base must outlive it).  The HyperPlonk full witness is
 * the concatenation of its columns (hyperplonk/src/proof/proof.rs:270); its
 * columns are views of it, so nothing is copied. */
int qg_buf_view(qg_buf* base, size_t offset, size_t n, qg_buf** out);
/* Upload n Montgomery Fr to entries [offset, offset+n). */
int qg_buf_upload_at(qg_buf* buf, size_t offset, const uint64_t* fr, size_t n);
/* Upload n canonical (non-Montgomery) 4 x u64 LE values < r, converted on the
 * device (QG_ERR_INVALID if some value >= r). */
int qg_buf_upload_canonical(qg_buf* buf, size_t offset, const uint64_t* canon, size_t n);
/* F::from(u64) for n values: the id / permutation index columns of
 * Circuit::permutation (hyperplonk/src/frontend/transition_circuit.rs:120-151). */
int qg_buf_upload_u64(qg_buf* buf, size_t offset, const uint64_t* v, size_t n);
/* Device-to-device copy of n entries. */
int qg_buf_copy(qg_buf* dst, size_t dst_off, const qg_buf* src, size_t src_off, size_t n);
/* First i < n with a[a_off+i] != b[b_off+i], or -1: the copy-constraint check
 * of TransitionCircuit::check_constraints (transition_circuit.rs:186-202). */
int qg_buf_first_mismatch(const qg_buf* a, size_t a_off, const qg_buf* b, size_t b_off, size_t n,
                          int64_t* first);

/* ---------------------------------------------------------------- MSM / KZG */
/* E::G1::msm_unchecked(bases, scalars) (pcs/src/kzg.rs:72): sum of
 * scalars[i] * srs[i] over i < n (n <= qg_srs_len).  Bit-exact: the affine
 * result is the unique group element. */
int qg_msm_g1(qg_ctx* ctx, const qg_srs* srs, const uint64_t* scalars, size_t n,
              uint64_t out_xy[8], uint8_t* out_inf);
int qg_msm_g1_dev(qg_ctx* ctx, const qg_srs* srs, const qg_buf* scalars, size_t n,
                  uint64_t out_xy[8], uint8_t* out_inf);
/* msm_unchecked over the base slice srs[offset..] (SURVEY 8(b)'s `offset`):
 * sum of scalars[i] * srs[offset + i] over i < min(n, qg_srs_len - offset),
 * truncated like msm_unchecked; QG_ERR_INVALID when offset > qg_srs_len.
 * Host (`_at`) and device-resident (`_dev_at`) scalars. */
int qg_msm_g1_at(qg_ctx* ctx, const qg_srs* srs, size_t offset, const uint64_t* scalars,
                 size_t n, uint64_t out_xy[8], uint8_t* out_inf);
int qg_msm_g1_dev_at(qg_ctx* ctx, const qg_srs* srs, size_t offset, const qg_buf* scalars,
                     size_t n, uint64_t out_xy[8], uint8_t* out_inf);
/* k MSMs over one SRS in one call (at most 1024): out_xy[8 i ..], out_inf[i]
 * for scalars[i] (first ns[i] entries), each equal to qg_msm_g1_dev of it.
 * They run as one MSM batch (bucketing beside the previous MSM's accumulation
 * on two side streams, one set of reduction launches): the commitments a
 * caller needs together, e.g. HyperPlonk's two Logup denominator columns
 * (multiset_check.rs:43-95) or its trace witnesses (proof.rs:252-262). */
int qg_msm_g1_dev_batch(qg_ctx* ctx, const qg_srs* srs, const qg_buf* const* scalars,
                        const size_t* ns, size_t k, uint64_t* out_xy, uint8_t* out_inf);
/* KZG::commit (kzg.rs:61-73): QG_ERR_INVALID when n > max_degree + 1
 * (reference: assert! at kzg.rs:62-65). */
int qg_kzg_commit(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                  uint64_t out_xy[8], uint8_t* out_inf);

/* KZGOpeningProof (kzg.rs:25-32). */
typedef struct qg_kzg_opening {
  uint64_t x[4];
  uint64_t y[4];
  uint64_t proof_xy[8];
  uint8_t proof_inf;
  uint8_t _pad[7];
} qg_kzg_opening;

/* KZG::open (kzg.rs:75-96): y = p(x), q = (p - y)/(X - x), proof = commit(q). */
int qg_kzg_open(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                const uint64_t x[4], qg_kzg_opening* out);

/* ---------------------------------------------------------------- multilinear PCS */
/* MLEvalProof (pcs/src/mlpcs.rs:32-44) without the point (caller owns it). */
typedef struct qg_mle_proof {
  uint64_t evaluation[4];
  uint64_t s_comm_xy[8];
  uint8_t s_comm_inf;
  uint8_t _pad[7];
  qg_kzg_opening poly_opening;
  qg_kzg_opening poly_opening_inv;
  qg_kzg_opening s_opening;
  qg_kzg_opening s_opening_inv;
} qg_mle_proof;

/* MultilinearPCS::open == MLEvalProof::prove (mlpcs.rs:83-124, trait impl
 * :191-198): opens the hypercube evaluations `poly` (len n) at `point`
 * (nvars Fr).  `state` is the transcript, advanced exactly as the reference
 * (append point, evaluation, s_comm; draw r). */
int qg_mle_open(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                const uint64_t* point, size_t nvars, uint8_t state[32], qg_mle_proof* out);
/* Same, on a device-resident evaluation vector (first n entries of `poly`). */
int qg_mle_open_dev(qg_ctx* ctx, const qg_srs* srs, const qg_buf* poly, size_t n,
                    const uint64_t* point, size_t nvars, uint8_t state[32], qg_mle_proof* out);
/* Same, with flags.  QG_OPEN_UNCHANGED: the caller guarantees that the first n
 * entries of `poly` have not changed since an earlier open of this same buffer
 * on this context; the polynomial's NTT transform from that call is then
 * reused when the context still holds it (HyperPlonk opens its full witness
 * once per column, proof.rs:203-224).  The proof is identical either way. */
#define QG_OPEN_UNCHANGED 1u
int qg_mle_open_dev_ex(qg_ctx* ctx, const qg_srs* srs, const qg_buf* poly, size_t n,
                       const uint64_t* point, size_t nvars, uint8_t state[32], uint32_t flags,
                       qg_mle_proof* out);
/* K openings in one call (at most 256), item k exactly as the k-th of K
 * successive qg_mle_open_dev_ex calls on the same transcript: same proofs, same
 * final `state`.  The S polynomial, its commitment and the evaluation depend
 * on (poly, point) only and no quotient commitment enters the transcript
 * (mlpcs.rs:83-124), so the device runs the K S commitments as one MSM batch,
 * the K transcript steps on the host, then all 4K quotient commitments as one
 * MSM batch.  HyperPlonk's openings of one trace (proof.rs:203-224).
 * HBM: the call holds every item's S (M - 1 Fr) and four quotient vectors
 * plus one partial-sum slot set per MSM until it returns (~1 GB per item of
 * 2^20 evaluations, mostly the partial slots); per-item scratch beyond the
 * first 16 items is freed when it returns, the first 16 items' is kept for
 * the next call.  A sharded
 * context (qg_ctx_attach_comm) batches too: all items must then share one SRS
 * shard (the Python mirror batches each run of equal local length). */
typedef struct qg_mle_open_item {
  const qg_buf* poly;     /* device evaluations (first n entries) */
  size_t n;
  const uint64_t* point;  /* nvars Fr */
  size_t nvars;
  uint32_t flags;         /* QG_OPEN_UNCHANGED or 0 */
  uint32_t _pad;
} qg_mle_open_item;
int qg_mle_open_batch_dev(qg_ctx* ctx, const qg_srs* srs, const qg_mle_open_item* items,
                          size_t k, uint8_t state[32], qg_mle_proof* outs);

/* ---------------------------------------------------------------- verifiers (host) */
/* BN254 G2 affine points on the D-type twist E'/Fq2 (y^2 = x^3 + 3/(9 + u)):
 * x.c0, x.c1, y.c0, y.c1, each 4 u64 Montgomery limbs (like G1's Fq). */
/* the standard generator (ark-bn254's G2Affine::generator()) */
int qg_g2_generator(uint64_t out_xy[16]);
/* k * Q (k: Fr, Montgomery limbs) — builds g2_points[1] = tau g2 of
 * KZG::trusted_setup (kzg.rs:52-53).  QG_ERR_INVALID off the curve or
 * outside the prime-order subgroup ([r] Q != O; ark's Validate::Yes). */
int qg_g2_mul(const uint64_t xy[16], uint8_t inf, const uint64_t k[4], uint64_t out_xy[16],
              uint8_t* out_inf);
/* The reduced optimal-ate pairing used by E::pairing (called at
 * kzg.rs:104-105): f_{6x+2,Q}(P) with Frobenius lines, raised to
 * (p^12 - 1) / r, in Fq12 = Fq6[w]/(w^2 - v), Fq6 = Fq2[v]/(v^3 - (9 + u));
 * out = c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2, each (re, im), Montgomery.
 * Guaranteed: bilinear, non-degenerate, of order r, so every GT equality
 * (KZG / ML-PCS verification equations) holds exactly when it does with
 * ark-bn254.  NOT guaranteed: the raw GT value equals ark-bn254's
 * `E::pairing(P, Q).0` — ark's hard-part addition chain may return a fixed
 * power of this value (parity of raw values with ark is unpinned; compare
 * GT elements only with each other).  G2 inputs must be on the twist and in
 * the prime-order subgroup (QG_ERR_INVALID otherwise). */
int qg_pairing(const uint64_t p_xy[8], uint8_t p_inf, const uint64_t q_xy[16], uint8_t q_inf,
               uint64_t out[48]);
/* The verifier's view of KZG (kzg.rs:10-23): g1, g2 = g2_points[0],
 * g2_tau = g2_points[1]. */
typedef struct qg_kzg_vk {
  uint64_t g1_xy[8];
  uint64_t g2_xy[16];
  uint64_t g2_tau_xy[16];
} qg_kzg_vk;
/* KZG::verify (kzg.rs:98-108): *ok = e(C - y g1, g2) == e(proof, g2_tau - x g2). */
int qg_kzg_verify(const qg_kzg_vk* vk, const uint64_t comm_xy[8], uint8_t comm_inf,
                  const qg_kzg_opening* opening, int* ok);
/* MLEvalProof::verify (mlpcs.rs:126-161): replays the transcript (append
 * point, evaluation, s_comm; draw r), verifies the four openings and the
 * inner-product equation at r.  `state` advances exactly as the prover's. */
int qg_mle_verify(const qg_kzg_vk* vk, const uint64_t comm_xy[8], uint8_t comm_inf,
                  const uint64_t* point, size_t nvars, const qg_mle_proof* proof,
                  uint8_t state[32], int* ok);

/* Building blocks of the opening, exposed for testing and for callers that
 * batch their own protocol:
 *  compute_pr (mlpcs.rs:68-78) == eq(bin(i), point) table, untrimmed (2^nvars) */
int qg_eq_table(qg_ctx* ctx, const uint64_t* point, size_t nvars, uint64_t* out);
/*  fast_eq_eval_hypercube (hyperplonk/src/utils/eq_eval.rs:6-31) into a device
 *  vector (first 2^nvars entries of `out`).  With a communicator attached:
 *  this rank's block, the 2^(nvars - log2 world) entries whose high index bits
 *  equal the rank. */
int qg_eq_table_dev(qg_ctx* ctx, const uint64_t* point, size_t nvars, qg_buf* out);
/*  InnerProductProof::compute_s_polynomial (pcs/src/ipa.rs:122-157), untrimmed:
 *  out has max(nf, ng) - 1 entries (caller trims trailing zeros). */
int qg_s_polynomial(qg_ctx* ctx, const uint64_t* f, size_t nf, const uint64_t* g, size_t ng,
                    uint64_t* out);
/*  sum_i f[i] g[i] over min(nf, ng)  (mlpcs.rs:91-94, ipa.rs:66-69) */
int qg_inner_product(qg_ctx* ctx, const uint64_t* f, size_t nf, const uint64_t* g, size_t ng,
                     uint64_t out[4]);

/* ---------------------------------------------------------------- sumcheck */
/* Virtual-polynomial expression (hyperplonk/src/utils/virtual_polynomial.rs:9-18)
 * in postfix form: INPUT(i) pushes table i, CONST(c) pushes consts[c],
 * ADD / MUL pop two and push the result.  Sub is ADD(a, MUL(CONST(-1), b)) as
 * in the reference (:67-77). */
#define QG_OP_INPUT 0
#define QG_OP_CONST 1
#define QG_OP_ADD 2
#define QG_OP_MUL 3
typedef struct qg_expr_op {
  uint32_t op;
  uint32_t arg;
} qg_expr_op;

/* SumcheckProof::prove (hyperplonk/src/piops/sumcheck.rs:28-114) for
 * h(g_0..g_{k-1}) = program.  tables[i] = 2^nvars Fr evaluations of g_i
 * (host pointers).  With an attached communicator (qg_ctx_attach_comm),
 * `nvars` is the GLOBAL variable count and each rank passes its block of
 * 2^(nvars - log2(world)) entries per table (high index bits = rank); every
 * rank returns the same proof.  Absorbs num_vars and claimed_sum, then per round the
 * trimmed coefficient-form message; binds index bit 0 first.
 * Outputs (caller-allocated):
 *   round_coeffs : nvars * (max_degree+1) * 4 uint64, row j = message j
 *                  coefficients (trailing zeros trimmed, rest zero-filled)
 *   round_lens   : nvars uint32, trimmed length of each message
 *   point        : nvars Fr (the EvaluationClaim point)
 *   evaluation   : h at the point (EvaluationClaim::evaluation)
 * `max_degree` = the expression's syntactic degree (qg_expr_degree). */
int qg_expr_degree(const qg_expr_op* prog, size_t prog_len, uint32_t* out_degree);
int qg_sumcheck_prove(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                      const uint64_t* const* tables, const qg_expr_op* prog, size_t prog_len,
                      const uint64_t* consts, size_t nconsts, const uint64_t claimed_sum[4],
                      uint8_t state[32], uint64_t* round_coeffs, uint32_t* round_lens,
                      uint64_t* point, uint64_t evaluation[4]);
/* Same with device-resident tables (the caller's buffers are not modified). */
int qg_sumcheck_prove_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                          const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                          const uint64_t* consts, size_t nconsts, const uint64_t claimed_sum[4],
                          uint8_t state[32], uint64_t* round_coeffs, uint32_t* round_lens,
                          uint64_t* point, uint64_t evaluation[4]);
/* The caller's transcript stays authoritative (the callback
 * form of SumcheckProof::prove, sumcheck.rs:28-114, whose `transcript:
 * &mut Transcript` is any implementation).  Per round j the library computes
 * the trimmed coefficient-form message and calls
 *   challenge(user, coeffs, len, out_r)
 * with `len` coefficients (len x 4 uint64, arkworks' in-memory Montgomery
 * limbs; len = 0 for an all-zero message); the callback appends the message
 * to its transcript (append_serializable of the DensePolynomial,
 * sumcheck.rs:80), draws r_j (draw_field_element, :82) and writes it to out_r
 * (Montgomery limbs); a nonzero return aborts the prove (QG_ERR_INVALID).
 * The caller appends num_vars and claimed_sum itself before the call
 * (sumcheck.rs:35-36); `claimed_sum` is not absorbed here.  Device tables,
 * any expression (the interpreted path; one host round trip per round), and
 * on a sharded context every rank calls its own callback (the ranks' replicas
 * must return the same r_j).  Outputs as qg_sumcheck_prove. */
typedef int (*qg_challenge_fn)(void* user, const uint64_t* coeffs, uint32_t len, uint64_t out_r[4]);
int qg_sumcheck_prove_cb(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                         const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                         const uint64_t* consts, size_t nconsts, qg_challenge_fn challenge,
                         void* user, uint64_t* round_coeffs, uint32_t* round_lens,
                         uint64_t* point, uint64_t evaluation[4]);

/* ZeroCheckProof::prove (hyperplonk/src/piops/zerocheck.rs:14-49): draws
 * z (nvars challenges), builds eq(., z) on the device (eq_eval.rs:6-31),
 * runs the sumcheck of h * eq with claimed sum 0 and returns the zero-check
 * claim evaluation = sumcheck claim / eq(z, point).  If `eq_out` is not NULL
 * it receives the eq table (2^nvars Fr) so the caller can mirror the store
 * mutation of zerocheck.rs:27-29.  Outputs as qg_sumcheck_prove, with
 * round messages of degree max_degree(h) + 1. */
int qg_zerocheck_prove(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                       const uint64_t* const* tables, const qg_expr_op* prog, size_t prog_len,
                       const uint64_t* consts, size_t nconsts, uint8_t state[32],
                       uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                       uint64_t evaluation[4], uint64_t* eq_out);
int qg_zerocheck_prove_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                           const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                           const uint64_t* consts, size_t nconsts, uint8_t state[32],
                           uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                           uint64_t evaluation[4]);

/* ---------------------------------------------------------------- Logup */
/* Log-derivative column of the Logup PIOPs: the per-row loops of
 * MultisetEqualityProof::prove (hyperplonk/src/piops/multiset_check.rs:43-95)
 * and SetInclusionProof::prove (hyperplonk/src/piops/set_inclusion.rs:93-131):
 *     out[x] = m(x) / (beta + h(x))        for every row x of the hypercube,
 * h and m given as postfix expressions over `tables` (same encoding as the
 * sumcheck above; m = 1 when m_prog is NULL, LookupMode::Equality).  Rows are
 * 2^nvars (with a communicator attached: nvars is global and each rank passes
 * and receives its 2^(nvars - log2(world)) block).  `out_sum` (nullable)
 * receives sum_x out[x] over all ranks — the claimed sums of
 * set_inclusion.rs:162-166,193-197.  Returns QG_ERR_ASSERT when some
 * beta + h(x) == 0 (the reference panics in inverse().unwrap(), :51/:63);
 * on any error the contents of `out` are undefined (the reference aborts
 * there, so no caller reads it).
 * Limits: <= 128 monomials per expression, <= 64 distinct tables. */
int qg_logup_column(qg_ctx* ctx, uint32_t nvars, uint32_t ntables, const uint64_t* const* tables,
                    const qg_expr_op* h_prog, size_t h_len, const uint64_t* h_consts,
                    size_t h_nconsts, const qg_expr_op* m_prog, size_t m_len,
                    const uint64_t* m_consts, size_t m_nconsts, const uint64_t beta[4],
                    uint64_t* out, uint64_t out_sum[4]);
/* Same with device-resident tables and output (out must not alias a table). */
int qg_logup_column_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables, const qg_buf* const* tables,
                        const qg_expr_op* h_prog, size_t h_len, const uint64_t* h_consts,
                        size_t h_nconsts, const qg_expr_op* m_prog, size_t m_len,
                        const uint64_t* m_consts, size_t m_nconsts, const uint64_t beta[4],
                        qg_buf* out, uint64_t out_sum[4]);

/* Circuit::check_constraints for one constraint expression
 * (hyperplonk/src/frontend/transition_circuit.rs:153-172): `first_row`
 * receives the first row x of the hypercube (this rank's block) with
 * h(x) != 0, or -1 when h vanishes on every row. */
int qg_expr_first_nonzero_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                              const qg_buf* const* tables, const qg_expr_op* prog, size_t len,
                              const uint64_t* consts, size_t nconsts, int64_t* first_row);

/* ---------------------------------------------------------------- profiling */
/* Per-kernel device time (ms) of the last call on this context, measured with
 * HIP events on the stream the kernels run on.  `name` is one of the kernel
 * group names listed in DESIGN.md (e.g. "msm_accumulate", "sumcheck_round").
 * Returns total ms and the launch count. */
int qg_ctx_enable_timing(qg_ctx* ctx, int enable);
/* Device Fq Montgomery-multiplication throughput (multiplies per second) from
 * a dependent-chain microbenchmark saturating every CU: the compute roof the
 * MSM's 11-Fq-mult-per-add cost is priced against. */
int qg_microbench_fq_mul(qg_ctx* ctx, double* mul_per_s);
/* FETCH_SIZE calibration for the PMC traffic figures: `gathers` random
 * 128-B table-row gathers in k_msm_accumulate's load pattern (k_fetch_gather),
 * then one 16-B-per-lane streaming read of the whole rows x 128-B table
 * (k_fetch_stream); device ms of each.  Known byte counts for rocprofv3. */
int qg_microbench_fetch(qg_ctx* ctx, size_t rows, size_t gathers, double* gather_ms,
                        double* stream_ms);
int qg_ctx_kernel_time(const qg_ctx* ctx, const char* name, double* total_ms, uint32_t* launches);
/* Additive split of the device-busy time among the k phase names given (the
 * same groups as qg_ctx_kernel_time, timing on): every interval in which m of
 * the listed phases' regions are open - on any of the context's streams - is
 * split evenly among those m phases, so the k values sum to the time at least
 * one of them was running (<= the wall time), where qg_ctx_kernel_time's
 * per-stream spans overlap (an MSM batch's bucketing beside the other side
 * stream's accumulation).  busy_ms[i] receives the share of names[i]. */
int qg_ctx_phase_split(const qg_ctx* ctx, const char* const* names, size_t k, double* busy_ms);
/* Profiling marker: launches an empty kernel (k_trace_marker) of `tag` work-groups
 * on the context stream, so a rocprofv3 kernel trace can be cut into the
 * caller's phases (profiles/kstats.py --legs groups dispatches by the last
 * marker).  No other effect. */
int qg_trace_marker(qg_ctx* ctx, uint32_t tag);
/* Diagnostic counters of the context by name; unknown names give 0.
 * "msm_plan_refetch": MSM bucket-scan plan copies (pinned, event-ordered) that
 * did not carry their run's generation tag and were re-read synchronously.
 * "msm_handover_violation": MSM batches whose event-ordered hand-over between
 * the context stream and the side streams the device guard found unordered
 * (each was recomputed in stream order; 0 while the event ordering holds). */
int qg_ctx_counter(const qg_ctx* ctx, const char* name, uint64_t* value);
/* Self-test of the binary-GCD field inversion the Logup column uses per block
 * (csrc/bingcd.h): out[i] = in[i]^-1 (plain canonical integers, 4 x u64 LE;
 * 0 -> 0) in Fr (field = 0) or Fq (field = 1), on the host (ctx may be NULL)
 * or, with on_device, in a device kernel on ctx. */
int qg_selftest_inverse(qg_ctx* ctx, int field, int on_device, const uint64_t* in, uint64_t* out,
                        size_t n);

#ifdef __cplusplus
}
#endif
#endif /* QUILL_GPU_H */
