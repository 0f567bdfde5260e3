// Where the half-space tail's time goes: the parts of constraints.hpp::minkowski_cell timed
// separately on one C2-like cell (T = 8, 28 (t, tau) pairs, covariance in LDS), with
// s_memrealtime (100 MHz) inside the kernel.  Parts: 0 pair_moments, 1 + first MVOE, 2 + second
// MVOE, 3 minkowski_pair (+ tangent, record store), 4 lower bound, 5 minkowski_cell, 6 = 3
// with the record written to LDS.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../include -I../cc-mpc_amd/csrc
//   tail_parts.hip -o tail_parts
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "constraints.hpp"

using namespace ccmpc;

constexpr int T = 8, ROWS = 2 * T, P = T * (T - 1) / 2;

template <int PART>
__global__ void part_kernel(const double *cov_g, const double *mean_g, MinkParams mp,
                            unsigned long long *ticks, double *sink, int reps) {
  __shared__ double cov[ROWS * ROWS];
  __shared__ double mean[ROWS];
  __shared__ double ref[ROWS + 3];
  __shared__ double lb_s[P];
  __shared__ ccmpc_halfspace rec_lds[P];
  for (int i = threadIdx.x; i < ROWS * ROWS; i += blockDim.x) cov[i] = cov_g[i];
  for (int i = threadIdx.x; i < ROWS; i += blockDim.x) mean[i] = mean_g[i];
  for (int i = threadIdx.x; i < ROWS + 3; i += blockDim.x)
    ref[i] = i < ROWS ? mp.ref_traj[i] : mp.cell_risk[i - ROWS];
  __syncthreads();
  double acc = 0.0;
  for (int r = 0; r < reps; ++r) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (PART == 5) {
      minkowski_cell(cov, mean, T, 0, ref, ref[ROWS], ref[ROWS + 1], ref[ROWS + 2], mp, lb_s,
                     threadIdx.x, blockDim.x);
    } else if (threadIdx.x < P) {
      int t, tau;
      pair_of(threadIdx.x, t, tau);
      if (PART == 3 || PART == 6) {
        minkowski_pair(cov, mean, ref, ROWS, t, tau, ref[ROWS], ref[ROWS + 1], mp.R, mp.tol,
                       mp.maxiter, PART == 3 ? mp.out_rec + threadIdx.x : rec_lds + threadIdx.x);
        if (PART == 6) acc += rec_lds[threadIdx.x].d;
      } else {
        const PairMoments pm = pair_moments(cov, ROWS, t, tau);
        double v = pm.cov_infer.a + pm.cov_mu.d;
        if (PART == 4) v = pair_lower_bound(pm, ref[ROWS + 2]);
        if (PART >= 1 && PART <= 2) {
          double b1;
          M2 Q;
          compute_mvoe(scale(pm.cov_infer, ref[ROWS]), scale(pm.cov_mu, ref[ROWS + 1]), mp.tol,
                       mp.maxiter, b1, Q);
          v = Q.a + b1;
          if (PART == 2) {
            double b2;
            M2 QR;
            compute_mvoe(Q, M2{mp.R * mp.R, 0.0, 0.0, mp.R * mp.R}, mp.tol, mp.maxiter, b2, QR);
            v = QR.a + b2;
          }
        }
        acc += v;
      }
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) ticks[r] = t1 - t0;
  }
  sink[threadIdx.x] = acc;
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
  double *d_cov, *d_mean, *d_ref, *d_risk, *d_plo, *d_sink;
  ccmpc_halfspace *d_rec;
  unsigned long long *d_ticks;
  const int reps = 20;
  (void)hipMalloc(&d_cov, cov.size() * 8);
  (void)hipMalloc(&d_mean, ROWS * 8);
  (void)hipMalloc(&d_ref, ROWS * 8);
  (void)hipMalloc(&d_risk, 3 * 8);
  (void)hipMalloc(&d_plo, T * 8);
  (void)hipMalloc(&d_sink, 256 * 8);
  (void)hipMalloc(&d_rec, P * sizeof(ccmpc_halfspace));
  (void)hipMalloc(&d_ticks, reps * 8);
  (void)hipMemcpy(d_cov, cov.data(), cov.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_mean, mean.data(), ROWS * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_ref, ref.data(), ROWS * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_risk, risk, 3 * 8, hipMemcpyHostToDevice);
  MinkParams mp{d_ref, nullptr, d_risk, 3.4, 1e-8, 1000, d_rec, d_plo};
  const char *names[] = {"pair_moments", "+ mvoe1", "+ mvoe2", "minkowski_pair",
                         "lower bound", "minkowski_cell", "pair -> LDS rec"};
  auto run = [&](auto kernel, int part) {
    hipLaunchKernelGGL(kernel, dim3(1), dim3(256), 0, 0, d_cov, d_mean, mp, d_ticks, d_sink, reps);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> ticks(reps);
    (void)hipMemcpy(ticks.data(), d_ticks, reps * 8, hipMemcpyDeviceToHost);
    std::sort(ticks.begin() + 1, ticks.end());
    printf("%-16s first %5.2f us  min %5.2f us  median %5.2f us\n", names[part],
           ticks[0] / 100.0, ticks[1] / 100.0, ticks[reps / 2] / 100.0);
  };
  run(part_kernel<0>, 0);
  run(part_kernel<1>, 1);
  run(part_kernel<2>, 2);
  run(part_kernel<3>, 3);
  run(part_kernel<4>, 4);
  run(part_kernel<5>, 5);
  run(part_kernel<6>, 6);
  return 0;
}
