/*
 * olpe.h -- C-ABI of libolpe.so, the MI355X (gfx950) implementation of the
 * apf_step2 Gibbs/Metropolis-Hastings hot path of logan-pearce/olpefit.
 *
 * The reference has no FFI: its seam is the call sequence at
 * apf_step2.py:312-318 (build_analytical_model -> chi_squared -> accept_reject)
 * driven by the loop at :300-365, module-level functions reading the globals
 * xsize/ysize.  Each entry point below names the reference code it replaces.
 *
 * Conventions
 *  - Every int-returning call returns OLPE_OK (0) or a negative OLPE_E* code and
 *    never aborts; olpe_last_error() gives a thread-local message.
 *  - The caller owns every host buffer.  A context owns the device copies of the
 *    image / inverse-sigma map and of the walker ensemble (state, counters, RNG).
 *  - One context is bound to one HIP device (no CPU path: device < 0 or a host
 *    without a GPU is an error).  Calls on one context are not thread-safe;
 *    separate contexts (one per GPU) may be used concurrently.
 *  - Parameter vectors use the reference layout: P = 16 (nsrc 2,
 *    apf_step2.py:108) or 19 (nsrc 3, 3body/apf_step2_3body.py:266-288)
 *    proposable parameters followed by the chi^2 slot, PS = P + 1 doubles.
 */
#ifndef OLPE_H
#define OLPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OLPE_OK 0
#define OLPE_EINVAL (-1)  /* bad argument */
#define OLPE_EHIP (-2)    /* HIP runtime error / no GPU */
#define OLPE_ENOMEM (-3)  /* device allocation failed */
#define OLPE_ESTATE (-4)  /* call out of order (e.g. run before seeding) */
#define OLPE_ECOMM (-5)   /* RCCL error */
#define OLPE_EIO (-6)     /* file write failed */

#define OLPE_DTYPE_F32 0
#define OLPE_DTYPE_F64 1

#define OLPE_EVAL_EXACT 0 /* one exp per pixel-Gaussian, reference op order */
#define OLPE_EVAL_FAST 1  /* separable exps + cross-term recurrence (default) */

typedef struct olpe_ctx olpe_ctx;

/* Library version (major*10000 + minor*100 + patch). */
int olpe_version(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int olpe_device_count(int *count);
/* Free / total device memory of a HIP device (sizes a run's launches so that the
 * per-launch chain buffer fits; OLPE_EHIP without a GPU). */
int olpe_device_mem(int device, long long *free_bytes, long long *total_bytes);
/* PCI bus id ("dddd:bb:dd.f") of a HIP device into buf (len >= 16): a multi-process run
 * checks that its ranks' devices are distinct GPUs whatever each process sees as device
 * 0..n-1 (bench.py, one process per GPU).  Build-specific: no reference counterpart. */
int olpe_device_pci_id(int device, char *buf, int len);
/* Thread-local message describing the last error. */
const char *olpe_last_error(void);

/* Create a context for one N x N cutout.  Replaces the setup at apf_step2.py:160-237
 * (the environment knob OLPE_WPB, a tuning experiment, must be 8, 12 or 16 and fit the
 * LDS, else OLPE_EINVAL with the byte count):
 *   image      ny*nx row-major, float32 (image_dtype OLPE_DTYPE_F32, BITPIX -32) or
 *              float64; promoted to f64 exactly as ``data - model`` does (:135).
 *   pois2      |D| Poisson term squared, same dtype as image, rounded as the
 *              reference rounds it (``np.sqrt(np.abs(image))**2``, :207-210).
 *   readnoise2 readnoise**2 (f64), :197-204.  err = sqrt(readnoise2 + pois2) (:210).
 *   mask       u8, 1 = excluded (``np.ma.masked_greater(image, 0.8*satlevel)``, :188);
 *              may be NULL (nothing masked).
 *   ny == nx   the reference is square-only (:237 swaps the axes and :123 fails to
 *              broadcast otherwise); ny != nx is OLPE_EINVAL.
 *   nsrc       2 (apf_step2.py) or 3 (3body/apf_step2_3body.py).
 *   bkgd_mode  0 = reference quirk, background fill p[12] (apf_step2.py:119-120);
 *              1 = fill p[9] (the dead code at :126-132).  Ignored for nsrc 3.
 *   device     HIP ordinal (>= 0). */
int olpe_create(const void *image, int image_dtype, const void *pois2, double readnoise2,
                const uint8_t *mask, int ny, int nx, int nsrc, int bkgd_mode, int device,
                olpe_ctx **out);
void olpe_destroy(olpe_ctx *ctx);
/* Select OLPE_EVAL_FAST (default) or OLPE_EVAL_EXACT for every evaluation of ctx. */
int olpe_set_eval_mode(olpe_ctx *ctx, int mode);

/* build_analytical_model (apf_step2.py:106-124; 3body :106-125): one PS-vector ->
 * N*N f64 model image.  Test hook. */
int olpe_model(olpe_ctx *ctx, const double *params, double *model_out);
/* chi_squared(image_nanmask, build_analytical_model(p), err) (apf_step2.py:314-316,
 * :134-137) for W parameter vectors [W][PS] -> chi2_out[W]. */
int olpe_chi2_batch(olpe_ctx *ctx, const double *params, int W, double *chi2_out);

/* --- walker ensemble (device resident) ------------------------------------------ */
/* np.random.seed(seeds[w]) for W walkers (init_genrand semantics)
 * and allocate the ensemble.  The reference seeds nothing (OS entropy per rank); the
 * build seeds per walker so runs are reproducible and GPU-count independent. */
int olpe_seed(olpe_ctx *ctx, const uint32_t *seeds, int W);
/* Upload walker state [W][PS] (params + chi^2) and counters tries/accepts [W][P]
 * (apf_step2.py:273-289; counters as the reference's float arrays, :276).
 * tries/accepts may be NULL (zeros).  If chi^2 slots are NaN they are NOT recomputed:
 * call olpe_chi2_batch first, as :283-289 does. */
int olpe_state_set(olpe_ctx *ctx, const double *state, const double *tries,
                   const double *accepts);
int olpe_state_get(olpe_ctx *ctx, double *state, double *tries, double *accepts);
/* Run n_iters Gibbs iterations of every walker (the loop body apf_step2.py:300-333)
 * asynchronously on the context's stream.  The ensemble keeps a global iteration
 * count c; the state after iteration c is recorded when c >= burn_in and
 * (c - burn_in) % record_stride == 0 (apf_step2.py:342-351 with stride 1) into the
 * device chain buffer of this launch (read with olpe_chain_read).  record_stride 0
 * records nothing.  accept_min > 0 tracks, per walker, the first c at which every
 * parameter has been tried accept_min times (the loop condition :300); read it with
 * olpe_done_at.  *nrec_out (may be NULL) = rows recorded per walker by this launch.
 * n_iters per call must be < 2^31 (OLPE_EINVAL otherwise; split long runs). */
int olpe_run(olpe_ctx *ctx, long long n_iters, long long burn_in, int record_stride,
             long long accept_min, long long *nrec_out);
/* Copy the last launch's chain [W][nrec][PS] to the host (synchronises). */
int olpe_chain_read(olpe_ctx *ctx, double *chain_out);
/* Iteration count of the ensemble (iterations completed so far). */
int olpe_count(olpe_ctx *ctx, long long *count);
int olpe_count_reset(olpe_ctx *ctx, long long count);
/* Per walker: first count c with min(tries) >= accept_min, or -1. */
int olpe_done_at(olpe_ctx *ctx, long long *done_at);
/* One-shot form of the loop: upload state/tries/accepts for W
 * walkers (already seeded with olpe_seed), reset the count to 0, run, download.
 * chain_out [W][nrec][PS] may be NULL. */
int olpe_run_gibbs(olpe_ctx *ctx, double *state, double *tries, double *accepts, int W,
                   long long n_iters, long long burn_in, int record_stride,
                   double *chain_out);

/* RNG state for resume/parity: mt_state [W][625] = 624 key words + position,
 * gauss_cache [W][2] = {has_gauss, cached deviate}. */
int olpe_rng_get(olpe_ctx *ctx, uint32_t *mt_state, double *gauss_cache);
int olpe_rng_set(olpe_ctx *ctx, const uint32_t *mt_state, const double *gauss_cache);
/* Test hook: draw n values per walker from the ensemble streams.
 * kind 0 = raw u32 (out as uint32 [W][n]); 1 = rand() f64; 2 = gauss f64;
 * 3 = randint(0, P) as f64.  Advances the streams. */
int olpe_rng_stream(olpe_ctx *ctx, int kind, int n, void *out);

/* Per-iteration trace of the next olpe_run (test hook): on != 0 enables it.
 * olpe_trace_read: [W][n_iters][6] f64 = {r, proposed value, chi^2 proposal, dice,
 * p_accept, accepted}. */
int olpe_trace_enable(olpe_ctx *ctx, int on);
int olpe_trace_read(olpe_ctx *ctx, double *out);

/* Wait for the context's stream. */
int olpe_sync(olpe_ctx *ctx);
/* Duration (ms, HIP events on the launch stream) of the last sampler launch. */
int olpe_last_kernel_ms(olpe_ctx *ctx, double *ms);
/* Durations of the last n sampler launches (oldest first; n <= 64 and <= launches so
 * far): launches can be queued back to back and timed afterwards. */
int olpe_kernel_times(olpe_ctx *ctx, int n, double *ms_out);
/* Chunks per walker of the last sampler launch (1 = whole walkers; > 1 when the launch
 * cut each walker's iterations into chunks to fill the resident waves).
 * Results do not depend on it.  Build-specific: no reference counterpart. */
int olpe_last_units(olpe_ctx *ctx, int *units);
/* Chunk hand-offs that had to wait since the context was created: out[0] = waits,
 * out[1] = total wave-time spent waiting (ns).  Diagnostics; build-specific. */
int olpe_unit_stats(olpe_ctx *ctx, long long *out);

/* --- chain files (apf_step2.py:342-360; 3body/apf_step2_3body.py:381-399) ---------
 * Host-only (no GPU needed).  Rows are formatted as the reference's csv.writer writes
 * a list of float rows: repr() of each value (shortest round-trip digits, fixed
 * notation for decimal exponents -4..15, 'nan'/'inf'), ',' between fields, "\r\n"
 * after each row.  nan_row != 0 prepends the all-NaN row the reference seeds
 * total_parameters with (apf_step2.py:278-279). */
/* Format rows [nrows][ncols] into out (cap bytes; out may be NULL to query the size):
 * *len_out = bytes of the text. */
int olpe_csv_format(const double *rows, long long nrows, int ncols, int nan_row, char *out,
                    size_t cap, size_t *len_out);
/* Write nfiles chain files: file i gets chains[i][nrows][ncols] (the per-walker
 * {rank}_finalarray_mpi.csv), from `threads` writer threads (0 = one per core). */
int olpe_csv_write_chains(const char *const *paths, const double *chains, int nfiles,
                          long long nrows, int ncols, int nan_row, int threads);

/* Streaming form of the same files.  The reference rewrites each file every 10
 * iterations (apf_step2.py:355-360), so a killed run leaves its chains on disk; the
 * build appends each launch's rows instead: rows [0, nrows) of
 * chains[i][rows_per_file][ncols] are appended to file i (created if absent; no NaN
 * row -- write it first with olpe_csv_write_chains and nrows 0).  sizes_out [nfiles]
 * (may be NULL) receives each file's size in bytes after the append: a checkpoint
 * records it, and a resumed run truncates the file back to it. */
int olpe_csv_append_chains(const char *const *paths, const double *chains, int nfiles,
                           long long rows_per_file, long long nrows, int ncols, int threads,
                           long long *sizes_out);

/* Step 3's read of the same files (apf_step3.py:169-186: np.genfromtxt per walker
 * file, the walkers collated as columns).  olpe_csv_shape: *rows = non-blank lines,
 * *cols = fields of the first line (step 3 takes the length from walker 0's file).
 * olpe_csv_read_chains: nfiles files of nrows x ncols each, rows [skip, nrows) into
 * out[nrows - skip][nfiles][ncols] (skip = step 3's additional_burnin, :190-205), parsed
 * from `threads` threads (0 = one per core); values equal genfromtxt's bit for bit
 * (correctly rounded; empty field = NaN).  A file of another shape is OLPE_EINVAL
 * naming the file (the reference fails assigning it into its [length, ncor] arrays). */
int olpe_csv_shape(const char *path, long long *rows, int *cols);
int olpe_csv_read_chains(const char *const *paths, int nfiles, long long nrows, int ncols,
                         long long skip, double *out, int threads);

/* Step 2's acceptance files (apf_step2.py:362-365: str(total_accept / total_tries), NumPy's
 * print of a float64 array).  Host-only.  olpe_acceptance_write: file i gets
 * accepts[i][np] / tries[i][np] as NumPy prints it, from `threads` threads (0 = one per
 * core), for the rows NumPy prints in fixed notation (all values finite, the non-zero
 * ones in [1e-4, 1e8) within a factor 1000 of each other): done[i] = 1; done[i] = 0 for
 * the rows left to the caller (scientific notation, NaN).  olpe_acceptance_format: the
 * text for x[0..n) (*len_out = 0 when x is outside that range; out may be NULL to query
 * the size). */
int olpe_acceptance_format(const double *x, int n, char *out, size_t cap, size_t *len_out);
int olpe_acceptance_write(const char *const *paths, const double *accepts, const double *tries,
                          int nfiles, int np, int threads, unsigned char *done);

/* --- multi-GPU (RCCL over xGMI), SURVEY.md §8(e) ---------------------------------
 * The reference's ranks meet at a per-iteration comm.barrier() (apf_step2.py:338); the
 * build's ranks meet only in these end-of-run collectives.  No rank is left waiting:
 * every call first all-reduces a word set (shard sizes, ranges, local failures), and a
 * rank decides whether to enter the data collective only from that agreed verdict (a
 * rank whose words cannot reach the device sends a poisoned default that fails the
 * check everywhere); the moments summary runs both all-reduce rounds on every rank and
 * decides success from their summed status words.  A failure inside a collective (a dead
 * peer) is bounded by olpe_comm_timeout: a rank that waits longer aborts its
 * communicator (OLPE_ECOMM; later collectives OLPE_ESTATE until olpe_comm_init). */
/* 128-byte RCCL unique id, created on rank 0 and shared by the host. */
int olpe_comm_unique_id(uint8_t *id128);
/* Join the communicator (a non-blocking RCCL communicator: its later waits are bounded by
 * olpe_comm_timeout).  The set-up itself returns once every rank has arrived -- RCCL's
 * bootstrap, not boundable here -- so callers meet on their own host group, with a
 * timeout, to share the id first (bench.py).  RCCL's own rank count and rank are checked
 * against nranks / rank. */
int olpe_comm_init(olpe_ctx *ctx, const uint8_t *id128, int nranks, int rank);
/* Seconds a collective may wait for the other ranks before it aborts the communicator and
 * returns OLPE_ECOMM; 0 = no bound.  Default 600.  Build-specific. */
int olpe_comm_timeout(olpe_ctx *ctx, double seconds);
/* RCCL's own view of the communicator: ncclCommCount / ncclCommUserRank (OLPE_ESTATE
 * without one).  Build-specific. */
int olpe_comm_info(olpe_ctx *ctx, int *nranks, int *rank);
/* All-gather the walker states of every rank: out [nranks*W][PS] (rank-major; equal W
 * on every rank, checked). */
int olpe_comm_allgather_state(olpe_ctx *ctx, double *out);
/* Chain concatenation (north star: "RCCL all-gather over xGMI only for the final chain
 * concatenation"; the reference leaves one {rank}_finalarray_mpi.csv per MPI rank,
 * apf_step2.py:355-360): all-gather walkers [w0, w0+wn) of the last launch's chain
 * from every rank into out [nranks][wn][nrec][PS] (rank-major; host memory, or NULL to
 * leave the gathered range in the context's device buffer, e.g. to time the
 * collective alone).  Gathering a large ensemble range by range bounds both the device
 * receive buffer and the host buffer by the range.  *nrec_out (may be NULL) = nrec.
 * Every rank must call with the same range and have the same W and nrec (checked:
 * OLPE_EINVAL on every rank otherwise).  The receive buffer is allocated before that
 * check and its outcome travels with it: a rank that cannot allocate it (or whose
 * olpe_comm_gather_limit it exceeds) makes the call OLPE_ENOMEM on every rank. */
int olpe_comm_allgather_chain(olpe_ctx *ctx, long long w0, long long wn, double *out,
                              long long *nrec_out);
/* Byte limit of the chain gather's device receive buffer (nranks x range bytes; 0 = no
 * limit, the default): a memory budget for the gather, like bench.py's --gather-mib. */
int olpe_comm_gather_limit(olpe_ctx *ctx, long long bytes);
/* Posterior summary over every rank from the whole-run moments (olpe_moments_*): two
 * all-reduces (sum), the pooled mean first, then the deviations of the walkers' means
 * about it.  out[OLPE_MOMENTS_LEN(PS, P)] as for olpe_moments_summary, over all ranks'
 * walkers, with centre = the pooled mean (out[2 + k] / out[1]).  Every rank must have
 * folded the same number of rows (checked: OLPE_EINVAL on every rank otherwise); the
 * walker counts may differ (a sum needs no equal shards).
 * Without olpe_comm_init it summarises this context alone.  Every local allocation (and
 * the zeroing of unfolded moments) happens before the uniformity check and its failure
 * travels in it (OLPE_ENOMEM on every rank); past the check every rank enters both
 * all-reduces whatever happened locally, a failure summed into a status word, so all
 * ranks return an error together (this rank's own, or OLPE_ECOMM naming how many other
 * ranks failed) -- except a rank that fails only to read round 2's sums back, which
 * returns its own error while its peers succeed. */
int olpe_comm_allreduce_moments(olpe_ctx *ctx, double *out);

/* --- whole-run posterior moments ----------------------------
 * apf_step3.py reads every chain file (:169-186) to compute per-parameter means, sigmas
 * and the Gelman-Rubin PSRF / RC (:258-278).  Those need, per walker w and column k,
 * only the walker's mean and sum of squared deviations M2 over its rows, which the
 * device keeps for every row the walker recorded: the summary then needs neither the
 * chain files nor a chain gather.  Rows = what the chain files hold after step 3's
 * default additional_burnin = 1 (the NaN seed row) -- every recorded row. */
/* Fold the last launch's recorded rows into the running (mean, M2) of every walker and
 * column (async; once per launch: OLPE_ESTATE if this launch was folded already).
 * olpe_seed starts a new run (no rows folded). */
int olpe_moments_accumulate(olpe_ctx *ctx);
int olpe_moments_reset(olpe_ctx *ctx);
/* *n = rows folded per walker; mean / m2 [W][PS] (either may be NULL).  _set restores a
 * checkpoint (n = 0: nothing folded; mean / m2 may then be NULL). */
int olpe_moments_get(olpe_ctx *ctx, long long *n, double *mean, double *m2);
int olpe_moments_set(olpe_ctx *ctx, long long n, const double *mean, const double *m2);
/* Per-column sums over this context's walkers (no communication):
 *   out[0] = n rows per walker, out[1] = walkers W,
 *   out[2 + k]          = sum_w mean_w[k]                         (k < PS)
 *   out[2 + PS + k]     = sum_w M2_w[k]
 *   out[2 + 2*PS + k]   = sum_w (mean_w[k] - centre[k])^2         (0 if centre is NULL)
 *   out[2 + 3*PS + j]   = sum_w tries_w[j], out[2 + 3*PS + P + j] = sum_w accepts_w[j]
 *                                                                 (j < P, whole run)
 * Per-parameter mean = out[2+k] / W; step 3's np.std over all rows =
 * sqrt((out[2+PS+k] + n * out[2+2PS+k]) / (n W)) with centre = that mean; GR's within
 * term = out[2+PS+k] / (n W), its between sum = out[2+2PS+k] (step3.summary_from_moments). */
#define OLPE_MOMENTS_LEN(ps, np) (2 + 3 * (ps) + 2 * (np))
int olpe_moments_summary(olpe_ctx *ctx, const double *centre, double *out);

#ifdef __cplusplus
}
#endif
#endif /* OLPE_H */
