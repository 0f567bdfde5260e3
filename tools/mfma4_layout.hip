// Determines the lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950 empirically: A and B get
// distinct per-lane values, D is compared against candidate layouts.
// Build: hipcc -O3 --offload-arch=gfx950 mfma4_layout.hip -o mfma4_layout
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void probe(const double *a, const double *b, double *d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

int main() {
  double a[64], b[64], d[64];
  for (int l = 0; l < 64; ++l) {
    a[l] = 1.0 + l;            // distinct
    b[l] = 1.0 + 0.01 * l * l;  // distinct, not linear in l
  }
  double *da, *db, *dd;
  (void)hipMalloc(&da, 512);
  (void)hipMalloc(&db, 512);
  (void)hipMalloc(&dd, 512);
  (void)hipMemcpy(da, a, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, 512, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(da, db, dd);
  (void)hipMemcpy(d, dd, 512, hipMemcpyDeviceToHost);
  // candidate layouts: A[bl][i][k] at lane fa(i,k,bl), B[bl][k][j] at lane fb(k,j,bl),
  // D[bl][i][j] at lane fd(i,j,bl)
  struct Cand {
    const char *name;
    int (*fa)(int, int, int);
    int (*fb)(int, int, int);
    int (*fd)(int, int, int);
  };
  Cand cands[] = {
      {"A:i+4k+16b B:j+4k+16b D:j+4i+16b", [](int i, int k, int bl) { return i + 4 * k + 16 * bl; },
       [](int k, int j, int bl) { return j + 4 * k + 16 * bl; },
       [](int i, int j, int bl) { return j + 4 * i + 16 * bl; }},
      {"A:i+4k+16b B:j+4k+16b D:i+4j+16b", [](int i, int k, int bl) { return i + 4 * k + 16 * bl; },
       [](int k, int j, int bl) { return j + 4 * k + 16 * bl; },
       [](int i, int j, int bl) { return i + 4 * j + 16 * bl; }},
      {"A:4i+k+16b B:4j+k+16b D:j+4i+16b", [](int i, int k, int bl) { return 4 * i + k + 16 * bl; },
       [](int k, int j, int bl) { return 4 * j + k + 16 * bl; },
       [](int i, int j, int bl) { return j + 4 * i + 16 * bl; }},
      {"A:4i+k+16b B:4j+k+16b D:i+4j+16b", [](int i, int k, int bl) { return 4 * i + k + 16 * bl; },
       [](int k, int j, int bl) { return 4 * j + k + 16 * bl; },
       [](int i, int j, int bl) { return i + 4 * j + 16 * bl; }},
      {"A:i+4b+16k B:j+4b+16k D:j+4i+16b", [](int i, int k, int bl) { return i + 4 * bl + 16 * k; },
       [](int k, int j, int bl) { return j + 4 * bl + 16 * k; },
       [](int i, int j, int bl) { return j + 4 * i + 16 * bl; }},
      {"A:i+4b+16k B:j+4b+16k D:j+4b+16i", [](int i, int k, int bl) { return i + 4 * bl + 16 * k; },
       [](int k, int j, int bl) { return j + 4 * bl + 16 * k; },
       [](int i, int j, int bl) { return j + 4 * bl + 16 * i; }},
      {"A:i+4b+16k B:j+4b+16k D:i+4b+16j", [](int i, int k, int bl) { return i + 4 * bl + 16 * k; },
       [](int k, int j, int bl) { return j + 4 * bl + 16 * k; },
       [](int i, int j, int bl) { return i + 4 * bl + 16 * j; }},
  };
  for (auto &c : cands) {
    double err = 0;
    for (int bl = 0; bl < 4; ++bl)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double s = 0;
          for (int k = 0; k < 4; ++k) s += a[c.fa(i, k, bl)] * b[c.fb(k, j, bl)];
          err = fmax(err, fabs(s - d[c.fd(i, j, bl)]));
        }
    printf("%-40s max err %g%s\n", c.name, err, err < 1e-9 ? "   <== MATCH" : "");
  }
  printf("d[0..7] = ");
  for (int l = 0; l < 8; ++l) printf("%g ", d[l]);
  printf("\n");
  return 0;
}
