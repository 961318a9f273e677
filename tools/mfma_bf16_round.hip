// Probe: how v_mfma_f32_16x16x32_bf16 rounds when it adds 32 bf16 x bf16 products to an f32
// accumulator.  One wave per case; every (m, n) of the tile gets C + sum_k a_k b_k (A rows and
// B columns identical), lane 0 writes D[0][0].  Host side: cases built from exact bf16 values,
// the exact sum in float64 and the f32 values the candidate rounding rules give.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(const uint16_t* a, const uint16_t* b, const float* c, float* out) {
  const int cs = blockIdx.x, l = threadIdx.x, g = l >> 4;
  uint16_t av[8], bv[8];
  for (int i = 0; i < 8; ++i) {
    av[i] = a[cs * 32 + 8 * g + i];
    bv[i] = b[cs * 32 + 8 * g + i];
  }
  bf8 A, B;
  memcpy(&A, av, 16);
  memcpy(&B, bv, 16);
  f4 C = f4{c[cs], c[cs], c[cs], c[cs]};
  f4 D = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, C, 0, 0, 0);
  if (l == 0) out[cs] = D[0];
}

static uint16_t bf(float x) {  // exact: callers pass bf16-representable values
  uint32_t u;
  memcpy(&u, &x, 4);
  if (u & 0xffff) { fprintf(stderr, "not a bf16: %g\n", x); exit(1); }
  return (uint16_t)(u >> 16);
}

struct Case { const char* name; float c; std::vector<float> a, b; };

int main() {
  std::vector<Case> cs;
  auto fill = [](float v, int n) { std::vector<float> x(32, 0.f); for (int i = 0; i < n; ++i) x[i] = v; return x; };
  const float one = 1.f;
  // single product p below / above half an ulp of C = 1 (ulp 2^-23)
  for (int k = 22; k <= 30; ++k) {
    for (float s : {1.f, -1.f}) {
      Case q{"", one, fill(0.f, 0), fill(0.f, 0)};
      q.a[0] = s * ldexpf(1.5f, -k);
      q.b[0] = 1.f;
      cs.push_back(q);
    }
  }
  // 32 equal products of 2^-k each (sum 2^(5-k)) added to C = 1
  for (int k = 24; k <= 34; ++k)
    for (float s : {1.f, -1.f}) cs.push_back(Case{"", one, fill(s * ldexpf(1.f, -k), 32), fill(1.f, 32)});
  // the products alone (C = 0): 1 + 31 tiny ones
  for (int k = 20; k <= 34; k += 2) {
    Case q{"", 0.f, fill(ldexpf(1.f, -k), 32), fill(1.f, 32)};
    q.a[0] = 1.f;
    cs.push_back(q);
    Case r{"", 0.f, fill(-ldexpf(1.f, -k), 32), fill(1.f, 32)};
    r.a[0] = 1.f;
    cs.push_back(r);
  }
  const int n = (int)cs.size();
  std::vector<uint16_t> ha(32 * n), hb(32 * n);
  std::vector<float> hc(n), ho(n);
  for (int i = 0; i < n; ++i) {
    hc[i] = cs[i].c;
    for (int k = 0; k < 32; ++k) { ha[32 * i + k] = bf(cs[i].a[k]); hb[32 * i + k] = bf(cs[i].b[k]); }
  }
  uint16_t *da, *db; float *dc, *dout;
  hipMalloc(&da, ha.size() * 2); hipMalloc(&db, hb.size() * 2); hipMalloc(&dc, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, 0, da, db, dc, dout);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
  hipMemcpy(ho.data(), dout, n * 4, hipMemcpyDeviceToHost);
  printf("case c a0 a1(=a_k,k>0) exact_f64 rne_f32 mfma mfma-exact(ulps of 1)\n");
  for (int i = 0; i < n; ++i) {
    double ex = cs[i].c;
    for (int k = 0; k < 32; ++k) ex += (double)cs[i].a[k] * cs[i].b[k];
    printf("%3d c=%g a0=%.9g a1=%.9g exact=%.17g rne=%.9g mfma=%.9g diff_ulp1=%.4f\n", i, cs[i].c, cs[i].a[0], cs[i].a[1],
           ex, (double)(float)ex, ho[i], (ho[i] - ex) / ldexp(1.0, -23));
  }
  return 0;
}
