// Microbenchmark of the half-space tail (constraints.hpp::minkowski_cell) on one C2-like cell:
// 2222 random-walk particles, T = 8, 28 (t, tau) pairs on one wave, covariance in LDS as the
// fused kernel has it.  Times the tail with s_memrealtime (100 MHz) inside the kernel, so
// launch overhead is excluded.  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -I../include -I../cc-mpc_amd/csrc pair_bench.hip -o pair_bench
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "constraints.hpp"

using namespace ccmpc;

constexpr int T = 8, ROWS = 2 * T, P = T * (T - 1) / 2;

__global__ void tail_kernel(const double *cov_g, const double *mean_g, MinkParams mp,
                            unsigned long long *ticks, int reps, int skip) {
  __shared__ double cov[ROWS * ROWS];
  __shared__ double mean[ROWS];
  __shared__ double ref[ROWS + 3];
  __shared__ double lb_s[P];
  for (int i = threadIdx.x; i < ROWS * ROWS; i += blockDim.x) cov[i] = cov_g[i];
  for (int i = threadIdx.x; i < ROWS; i += blockDim.x) mean[i] = mean_g[i];
  for (int i = threadIdx.x; i < ROWS + 3; i += blockDim.x)
    ref[i] = i < ROWS ? mp.ref_traj[i] : mp.cell_risk[i - ROWS];
  __syncthreads();
  for (int r = 0; r < reps; ++r) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    (void)skip;
    minkowski_cell(cov, mean, T, 0, ref, ref[ROWS], ref[ROWS + 1], ref[ROWS + 2], mp, lb_s,
                   threadIdx.x, blockDim.x);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) ticks[r] = t1 - t0;
    __syncthreads();
  }
}

int main() {
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd(0.0, 1.0);
  const int N = 2222;
  std::vector<double> x(static_cast<size_t>(N) * ROWS);
  for (int p = 0; p < N; ++p) {
    double px = 190.0, py = -80.0, vx = 2.0 + 0.3 * nd(rng), vy = 0.3 + 0.2 * nd(rng);
    for (int t = 0; t < T; ++t) {
      vx += 0.2 * nd(rng);
      vy += 0.2 * nd(rng);
      px += vx;
      py += vy;
      x[p * ROWS + 2 * t] = px;
      x[p * ROWS + 2 * t + 1] = py;
    }
  }
  std::vector<double> mean(ROWS, 0.0), cov(ROWS * ROWS, 0.0);
  for (int p = 0; p < N; ++p)
    for (int i = 0; i < ROWS; ++i) mean[i] += x[p * ROWS + i] / N;
  for (int p = 0; p < N; ++p)
    for (int i = 0; i < ROWS; ++i)
      for (int j = 0; j < ROWS; ++j)
        cov[i * ROWS + j] += (x[p * ROWS + i] - mean[i]) * (x[p * ROWS + j] - mean[j]) / (N - 1);
  std::vector<double> ref(ROWS);
  for (int t = 0; t < T; ++t) {
    ref[2 * t] = 170.0 + 4.0 * (t + 1);
    ref[2 * t + 1] = -70.0 + 0.5 * (t + 1);
  }
  const double eps = 0.05 / 4 / T;
  const double risk[3] = {-2.0 * std::log(eps), -2.0 * std::log(1e-4), 2.6};

  double *d_cov, *d_mean, *d_ref, *d_risk, *d_plo;
  ccmpc_halfspace *d_rec;
  unsigned long long *d_ticks;
  const int reps = 20;
  (void)hipMalloc(&d_cov, cov.size() * 8);
  (void)hipMalloc(&d_mean, ROWS * 8);
  (void)hipMalloc(&d_ref, ROWS * 8);
  (void)hipMalloc(&d_risk, 3 * 8);
  (void)hipMalloc(&d_plo, T * 8);
  (void)hipMalloc(&d_rec, P * sizeof(ccmpc_halfspace));
  (void)hipMalloc(&d_ticks, reps * 8);
  (void)hipMemcpy(d_cov, cov.data(), cov.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_mean, mean.data(), ROWS * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_ref, ref.data(), ROWS * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_risk, risk, 3 * 8, hipMemcpyHostToDevice);
  for (int maxiter : {1000, 1}) {
  MinkParams mp{d_ref, nullptr, d_risk, 3.4, 1e-8, maxiter, d_rec, d_plo};
  printf("maxiter=%d\n", maxiter);
  for (int threads : {64, 128, 256}) {
    const int skip = 0;
    hipLaunchKernelGGL(tail_kernel, dim3(1), dim3(threads), 0, 0, d_cov, d_mean, mp, d_ticks,
                       reps, skip);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> ticks(reps);
    (void)hipMemcpy(ticks.data(), d_ticks, reps * 8, hipMemcpyDeviceToHost);
    std::sort(ticks.begin() + 1, ticks.end());
    printf("threads=%3d: tail first %.2f us, min %.2f us, median %.2f us\n", threads,
           ticks[0] / 100.0, ticks[1] / 100.0, ticks[reps / 2] / 100.0);
  }
  }
  std::vector<ccmpc_halfspace> rec(P);
  (void)hipMemcpy(rec.data(), d_rec, P * sizeof(ccmpc_halfspace), hipMemcpyDeviceToHost);
  int bad = 0;
  double bsum = 0;
  for (auto &h : rec) {
    bad += h.status != 0;
    bsum += h.beta1 + h.beta2;
  }
  printf("records: %d non-ok, sum(beta) = %.17g, d[0] = %.17g\n", bad, bsum, rec[0].d);
  return 0;
}
