// bann_io_dev.hip — BedVM::from_file (io/bed.rs:193-245) onto the device: the
// .bed signature is checked (variant-major only, as the reference), the dims
// come from stem.dims or the .fam/.bim line counts, and the payload streams from
// the file through a bounded pinned block into the 2-bit genotype image
// (kernels_data.hip) -- the file is never held whole in host memory.
#include <stdio.h>

#include <algorithm>
#include <string>

#include "ctx_internal.h"

extern "C" int bann_genotypes_load_bed(bann_ctx* ctx, const char* stem) {
  if (!ctx || !stem) return BANN_E_ARG;
  int64_t n = 0, M = 0;
  if (bann_bed_dims(stem, &n, &M) != BANN_OK) return fail(ctx, BANN_E_ARG, "no .dims or .fam/.bim next to the .bed");
  const std::string path = std::string(stem) + ".bed";
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return fail(ctx, BANN_E_ARG, "cannot open " + path);
  unsigned char sig[3] = {0, 0, 0};
  if (fread(sig, 1, 3, f) != 3 || sig[0] != 0x6c || sig[1] != 0x1b || (sig[2] != 0x00 && sig[2] != 0x01)) {
    fclose(f);
    return fail(ctx, BANN_E_ARG, "unexpected .bed signature (bed.rs:104-117)");
  }
  if (sig[2] == 0x00) {
    fclose(f);
    return fail(ctx, BANN_E_ARG, "sample-major .bed is not supported (bed.rs:200-202)");
  }
  int rc = alloc_genotypes(ctx, n, M);
  if (rc) {
    fclose(f);
    return rc;
  }
  const int64_t bpc = (n + 3) / 4;
  const int64_t blk = stage_markers(bpc, M);
  uint8_t *h = nullptr, *d = nullptr;
  if (hipHostMalloc((void**)&h, (size_t)(blk * bpc), hipHostMallocDefault) != hipSuccess || dalloc(&d, blk * bpc)) {
    fclose(f);
    if (h) (void)hipHostFree(h);
    return fail(ctx, BANN_E_OOM, "staging buffers");
  }
  for (int64_t j0 = 0; j0 < M && rc == BANN_OK; j0 += blk) {
    const int64_t m = std::min(blk, M - j0);
    if (fread(h, 1, (size_t)(m * bpc), f) != (size_t)(m * bpc)) {
      rc = fail(ctx, BANN_E_SHAPE, ".bed payload shorter than the dims announce");
      break;
    }
    if (hipMemcpyAsync(d, h, (size_t)(m * bpc), hipMemcpyHostToDevice, ctx->stream) != hipSuccess) rc = BANN_E_HIP;
    launch_bed_to_raw(d, n, m, ctx->d_g + j0 * ctx->rowb, ctx->rowb, ctx->stream);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) rc = fail(ctx, BANN_E_HIP, "bed decode");  // h is reused
  }
  fclose(f);
  (void)hipHostFree(h);
  dfree(d);
  if (rc) return rc;
  launch_col_stats(ctx->d_g, ctx->rowb, ctx->d_mu, ctx->d_sigma, n, M, ctx->stream);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->stream));
  return BANN_OK;
}
