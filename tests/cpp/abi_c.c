/* Plain-C client of the drop-in boundary (include/hiccl_reduce.h): compiled
 * with gcc -std=c99 -pedantic by tests/test_abi.py, which proves the header
 * is C (no C++ in the signatures) and links against libhiccl_reduce.so.
 * Without an argument it runs only host-side checks (no GPU needed); with
 * "gpu" it reduces 3 device buffers of 1000 floats and compares with a host
 * loop in the reference's order (compute.h:14-23). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hiccl_reduce.h"

/* the few HIP runtime entry points the GPU leg needs, declared by hand so
 * this file needs nothing but the C ABI header and a C compiler */
extern int hipMalloc(void **p, size_t bytes);
extern int hipFree(void *p);
extern int hipMemcpy(void *dst, const void *src, size_t bytes, int kind);
extern int hipDeviceSynchronize(void);

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
      fails++;                                                \
    }                                                         \
  } while (0)

int main(int argc, char **argv) {
  const void *tab[2] = {(const void *)0x2000, (const void *)0x3000};
  hiccl_reduce_config_t cfg;
  hiccl_reduce_plan_t *plan = NULL;
  hiccl_host_pipe_t *pipe = NULL;
  CHECK(hiccl_dtype_size(HICCL_FLOAT32) == 4 && hiccl_dtype_size(HICCL_BFLOAT16) == 2);
  CHECK(hiccl_version() >= 100);
  CHECK(hiccl_reduce(99, (void *)0x1000, tab, 2, 4, NULL) != 0 && strstr(hiccl_last_error(), "dtype"));
  memset(&cfg, 0, sizeof(cfg));
  cfg.engine = 7;
  CHECK(hiccl_reduce_ex(HICCL_FLOAT32, (void *)0x1000, tab, 2, 4, NULL, &cfg) != 0);
  CHECK(hiccl_reduce_plan_create(&plan, 99, 0) != 0 && plan == NULL);
  CHECK(hiccl_host_pipe_create(&pipe, 99, 0, 0, 0) != 0 && pipe == NULL);
  hiccl_reduce_plan_destroy(NULL);
  hiccl_host_pipe_destroy(NULL);
  /* bucket layout: the stride rule and the host-side refusals */
  CHECK(hiccl_bucket_stride(HICCL_FLOAT32, (size_t)1 << 28) == ((size_t)1 << 30) + 65536);
  CHECK(hiccl_bucket_stride(99, 16) == 0);
  CHECK(hiccl_bucket_alloc(HICCL_FLOAT32, 2, 16, 0, NULL, NULL, NULL) != 0 && strstr(hiccl_last_error(), "NULL"));
  CHECK(hiccl_bucket_free(NULL) == 0);
  if (argc > 1 && strcmp(argv[1], "gpu") == 0) {
    enum { N = 3, COUNT = 1000 };
    float host[N][COUNT], out[COUNT];
    void *dev[N], *dout;
    const void *in[N];
    int k, i;
    for (k = 0; k < N; k++)
      for (i = 0; i < COUNT; i++) host[k][i] = (float)((i * 37 + k * 11) % 101) / 7.0f - 3.0f;
    for (k = 0; k < N; k++) {
      CHECK(hipMalloc(&dev[k], sizeof(host[k])) == 0);
      CHECK(hipMemcpy(dev[k], host[k], sizeof(host[k]), 1 /* hipMemcpyHostToDevice */) == 0);
      in[k] = dev[k];
    }
    CHECK(hipMalloc(&dout, sizeof(out)) == 0);
    CHECK(hiccl_reduce_f32((float *)dout, (const float *const *)in, N, COUNT, NULL) == 0);
    CHECK(hipDeviceSynchronize() == 0);
    CHECK(hipMemcpy(out, dout, sizeof(out), 2 /* hipMemcpyDeviceToHost */) == 0);
    for (i = 0; i < COUNT; i++) {
      float acc = 0.0f;
      for (k = 0; k < N; k++) acc += host[k][i];
      if (memcmp(&acc, &out[i], sizeof(float)) != 0) {
        fprintf(stderr, "element %d: %a != %a\n", i, (double)out[i], (double)acc);
        fails++;
        break;
      }
    }
    for (k = 0; k < N; k++) hipFree(dev[k]);
    hipFree(dout);
    { /* the same sum in a bucket (hiccl_bucket_alloc): same bits */
      void *base = NULL, *bin[N], *bout = NULL;
      float out2[COUNT];
      CHECK(hiccl_bucket_alloc(HICCL_FLOAT32, N, COUNT, 0, &base, bin, &bout) == 0);
      CHECK((char *)bin[1] - (char *)bin[0] == (ptrdiff_t)hiccl_bucket_stride(HICCL_FLOAT32, COUNT));
      for (k = 0; k < N; k++) CHECK(hipMemcpy(bin[k], host[k], sizeof(host[k]), 1) == 0);
      CHECK(hiccl_reduce(HICCL_FLOAT32, bout, (const void *const *)bin, N, COUNT, NULL) == 0);
      CHECK(hipDeviceSynchronize() == 0);
      CHECK(hipMemcpy(out2, bout, sizeof(out2), 2) == 0);
      CHECK(memcmp(out, out2, sizeof(out)) == 0);
      CHECK(hiccl_bucket_free(base) == 0);
    }
  }
  printf("abi_c: %s\n", fails ? "FAILED" : "PASSED");
  return fails ? 1 : 0;
}
