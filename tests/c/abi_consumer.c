/* A plain-C consumer of libolpe.so (include/olpe.h): no Python, no C++.  Built by
 * tests/test_c_consumer.py with gcc -std=c99 against the in-tree library.
 *
 *   abi_consumer csv                      host-only calls: version, device count, the
 *                                         chain-row formatter; prints what it got
 *   abi_consumer run <in.bin> <out.bin>   one-shot Gibbs run (olpe_run_gibbs, SURVEY.md
 *                                         §8(b)) of the walkers described by in.bin
 *
 * in.bin (little-endian): int32 n, nsrc, W, n_iters, mode; float64 readnoise2;
 * float32 image[n*n]; float32 pois2[n*n]; uint8 mask[n*n]; uint32 seeds[W];
 * float64 p0[PS] (chi^2 slot NaN: computed here).  out.bin: float64 state[W*PS], tries[W*P], accepts[W*P],
 * chain[W*n_iters*PS]. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "olpe.h"

static int fail(const char *what, int rc) {
  fprintf(stderr, "%s: rc %d: %s\n", what, rc, olpe_last_error());
  return 2;
}

static int read_all(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n; }

static int run(const char *in_path, const char *out_path) {
  FILE *f = fopen(in_path, "rb");
  if (!f) return fail("open input", -1);
  int32_t hdr[5];
  double rn2;
  if (!read_all(f, hdr, sizeof hdr) || !read_all(f, &rn2, sizeof rn2)) return fail("header", -1);
  const int n = hdr[0], nsrc = hdr[1], W = hdr[2], iters = hdr[3], mode = hdr[4];
  const int P = nsrc == 2 ? 16 : 19, PS = P + 1;
  const size_t npix = (size_t)n * n;
  float *image = malloc(npix * sizeof(float)), *pois2 = malloc(npix * sizeof(float));
  uint8_t *mask = malloc(npix);
  uint32_t *seeds = malloc((size_t)W * sizeof(uint32_t));
  double *p0 = malloc((size_t)PS * sizeof(double));
  if (!read_all(f, image, npix * sizeof(float)) || !read_all(f, pois2, npix * sizeof(float)) ||
      !read_all(f, mask, npix) || !read_all(f, seeds, (size_t)W * sizeof(uint32_t)) ||
      !read_all(f, p0, (size_t)PS * sizeof(double)))
    return fail("payload", -1);
  fclose(f);

  olpe_ctx *ctx = NULL;
  int rc = olpe_create(image, OLPE_DTYPE_F32, pois2, rn2, mask, n, n, nsrc, 0, 0, &ctx);
  if (rc) return fail("olpe_create", rc);
  if ((rc = olpe_set_eval_mode(ctx, mode))) return fail("olpe_set_eval_mode", rc);
  /* the initial chi^2 (apf_step2.py:283-289) through the batch entry point; the start
   * vector's own chi^2 slot is kept unless it is NaN (the caller's value, e.g. the
   * reference's, is what the first accept test compares against) */
  double chi = 0.0;
  if ((rc = olpe_chi2_batch(ctx, p0, 1, &chi))) return fail("olpe_chi2_batch", rc);
  if (p0[PS - 1] != p0[PS - 1]) p0[PS - 1] = chi;
  if ((rc = olpe_seed(ctx, seeds, W))) return fail("olpe_seed", rc);
  double *state = malloc((size_t)W * PS * sizeof(double));
  double *tries = calloc((size_t)W * P, sizeof(double));
  double *accepts = calloc((size_t)W * P, sizeof(double));
  double *chain = malloc((size_t)W * iters * PS * sizeof(double));
  for (int w = 0; w < W; ++w) memcpy(state + (size_t)w * PS, p0, (size_t)PS * sizeof(double));
  if ((rc = olpe_run_gibbs(ctx, state, tries, accepts, W, iters, 0, 1, chain)))
    return fail("olpe_run_gibbs", rc);
  olpe_destroy(ctx);

  FILE *o = fopen(out_path, "wb");
  if (!o) return fail("open output", -1);
  fwrite(state, sizeof(double), (size_t)W * PS, o);
  fwrite(tries, sizeof(double), (size_t)W * P, o);
  fwrite(accepts, sizeof(double), (size_t)W * P, o);
  fwrite(chain, sizeof(double), (size_t)W * iters * PS, o);
  fclose(o);
  printf("ran %d walkers x %d iterations (%s), initial chi2 %.17g\n", W, iters,
         mode == OLPE_EVAL_FAST ? "fast" : "exact", chi);
  free(image); free(pois2); free(mask); free(seeds); free(p0);
  free(state); free(tries); free(accepts); free(chain);
  return 0;
}

static int host_only(void) {
  int ndev = -1;
  if (olpe_device_count(&ndev)) return fail("olpe_device_count", -1);
  const double rows[2][3] = {{1.0, 0.1, -2.5e-7}, {12345678901234567.0, 1e16, 0.0}};
  size_t len = 0;
  int rc = olpe_csv_format(&rows[0][0], 2, 3, 1, NULL, 0, &len);
  if (rc) return fail("olpe_csv_format (size)", rc);
  char *buf = malloc(len + 1);
  if ((rc = olpe_csv_format(&rows[0][0], 2, 3, 1, buf, len, &len))) return fail("olpe_csv_format", rc);
  buf[len] = 0;
  printf("version %d\ndevices %d\n%s", olpe_version(), ndev, buf);
  free(buf);
  /* no CPU path: a context on a host without a GPU is an error, never a fallback */
  olpe_ctx *ctx = NULL;
  const float img[4] = {1, 2, 3, 4};
  rc = olpe_create(img, OLPE_DTYPE_F32, img, 1.0, NULL, 2, 2, 2, 0, 0, &ctx);
  printf("create rc %d%s\n", rc, ctx ? " ctx" : "");
  if (ctx) olpe_destroy(ctx);
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 2 && !strcmp(argv[1], "csv")) return host_only();
  if (argc >= 4 && !strcmp(argv[1], "run")) return run(argv[2], argv[3]);
  fprintf(stderr, "usage: %s csv | run <in.bin> <out.bin>\n", argv[0]);
  return 1;
}
