// metrics.hip — the evaluation path's spike metrics on the device:
//   src/trainer/base.py:180-198  exp of the log-rate predictions, then per session
//   src/utils/utils.py:122-181   metrics_list(gt^T, pred^T, ['bps', 'rsquared'])
//   src/utils/metric_utils.py:36-102  neg_log_likelihood / bits_per_spike
// Inputs are the session's concatenated eval tensors BEFORE base.py's transposes:
//   gt, pred [R trials, T bins, N neurons] f32 row-major (pred = rates, or log-rates with
//   log_input = 1, base.py:186's exp fused in, computed in f32 like torch.exp).
// bps (utils.py:125-134): for neuron c < n_eval (the reference loops over range(R) and indexes
//   the neuron axis with it — n_eval = R, R <= N checked by the host), with NaN spikes masked and
//   zero rates replaced by 1e-9 (metric_utils.py:60-73):
//     nll_model - nll_null = sum(r - n log r) - (cnt m - S log m),   m = S / cnt (the null model's
//     nanmean rate, 1e-9 if 0); the log(n!) terms of both likelihoods cancel exactly;
//     bps_c = (nll_null - nll_model) / S / ln 2, +-inf -> NaN; result = nanmean over c.
// rsquared (utils.py:153-167): for trial i, sklearn r2_score(y_true = gt[i]^T, y_pred) — samples
//   are the N neurons, outputs the T bins: per bin 1 - SS_res / SS_tot with sklearn's
//   force_finite rules (SS_res == 0 -> 1, SS_tot == 0 -> 0), uniform mean over bins, then the
//   NaN-ignoring mean over trials.  N < 2 gives NaN (sklearn's "less than two samples").
// Also mse / mae (utils.py:169-175) over all elements.  Everything accumulates in f64 in a fixed
// order (deterministic).  HBM-bound: one read of gt and pred per metric family.
#include <math.h>

#include "common.h"

namespace vs {

constexpr int kBpsStats = 6;  // cnt, S, sum r, sum n log r, #NaN rates, #negative rates
constexpr int kMaxChunks = 256;

__device__ __forceinline__ double rate_of(float x, int log_input) { return log_input ? (double)expf(x) : (double)x; }

// thread = neuron c, block-row = a chunk of the R*T rows; partials [chunk][stat][n_eval]
__global__ __launch_bounds__(256) void bps_partial_kernel(const float* __restrict__ gt, const float* __restrict__ pr,
                                                          int64_t rows, int64_t N, int64_t n_eval, int log_input,
                                                          int64_t rows_per_chunk, double* __restrict__ part) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= n_eval) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  double cnt = 0, S = 0, sr = 0, snl = 0, nnan = 0, nneg = 0;
  for (int64_t r = r0; r < r1; ++r) {
    const float y = gt[r * N + c];
    if (isnan(y)) continue;
    const double rate = rate_of(pr[r * N + c], log_input);
    if (isnan(rate)) {
      nnan += 1;
      continue;
    }
    if (rate < 0) {
      nneg += 1;
      continue;
    }
    const double rr = rate == 0.0 ? 1e-9 : rate;
    cnt += 1;
    S += y;
    sr += rr;
    snl += (double)y * log(rr);
  }
  double* p = part + (int64_t)blockIdx.y * kBpsStats * n_eval + c;
  p[0 * n_eval] = cnt;
  p[1 * n_eval] = S;
  p[2 * n_eval] = sr;
  p[3 * n_eval] = snl;
  p[4 * n_eval] = nnan;
  p[5 * n_eval] = nneg;
}

__global__ __launch_bounds__(256) void bps_neuron_kernel(const double* __restrict__ part, int chunks, int64_t n_eval,
                                                         double* __restrict__ bps, double* __restrict__ bad) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= n_eval) return;
  double st[kBpsStats] = {0, 0, 0, 0, 0, 0};
  for (int k = 0; k < chunks; ++k)
#pragma unroll
    for (int j = 0; j < kBpsStats; ++j) st[j] += part[((int64_t)k * kBpsStats + j) * n_eval + c];
  const double cnt = st[0], S = st[1];
  double v = __builtin_nan("");
  if (cnt > 0 && S != 0) {
    double m = S / cnt;
    if (m == 0) m = 1e-9;
    const double nll_null = cnt * m - S * log(m);
    const double nll_model = st[2] - st[3];
    v = (nll_null - nll_model) / S / 0.69314718055994530942;
    if (isinf(v)) v = __builtin_nan("");
  }
  bps[c] = v;
  bad[2 * c] = st[4];
  bad[2 * c + 1] = st[5];
}

// one wave per (trial, bin) row of N neurons: mean, SS_tot, SS_res (two passes over the row)
__global__ __launch_bounds__(256) void r2_row_kernel(const float* __restrict__ gt, const float* __restrict__ pr,
                                                     int64_t rows, int64_t N, int log_input, double* __restrict__ r2,
                                                     double* __restrict__ rowstat) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* y = gt + row * N;
  const float* x = pr + row * N;
  double sy = 0, nbad = 0;
  for (int64_t n = lane; n < N; n += 64) sy += y[n];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sy += __shfl_xor(sy, o, 64);
  const double mean = sy / (double)N;
  double tot = 0, res = 0, ab = 0;
  for (int64_t n = lane; n < N; n += 64) {
    const double yv = y[n], pv = rate_of(x[n], log_input);
    if (isnan(yv) || isnan(pv) || isinf(yv) || isinf(pv)) nbad += 1;  // sklearn rejects NaN / inf
    const double d = yv - pv, e = yv - mean;
    res += d * d;
    tot += e * e;
    ab += fabs(d);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    tot += __shfl_xor(tot, o, 64);
    res += __shfl_xor(res, o, 64);
    ab += __shfl_xor(ab, o, 64);
    nbad += __shfl_xor(nbad, o, 64);
  }
  if (lane == 0) {
    double v;
    if (N < 2) v = __builtin_nan("");
    else if (res == 0) v = 1.0;   // perfect prediction (even for a constant row)
    else if (tot == 0) v = 0.0;   // constant row, imperfect prediction
    else v = 1.0 - res / tot;
    r2[row] = v;
    rowstat[3 * row + 0] = nbad;
    rowstat[3 * row + 1] = res;
    rowstat[3 * row + 2] = ab;
  }
}

// fixed-shape block reductions (256 threads)
__device__ double block_sum(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double s = red[0];
  __syncthreads();
  return s;
}

// out: [0] bps, [1] rsquared, [2] #NaN rates, [3] #negative rates, [4] #NaN r2 inputs, [5] mse, [6] mae
__global__ __launch_bounds__(256) void metrics_final_kernel(const double* __restrict__ bps, const double* __restrict__ bad,
                                                            int64_t n_eval, const double* __restrict__ r2,
                                                            const double* __restrict__ rowstat, int64_t R, int64_t T,
                                                            int64_t N, int do_r2, double* __restrict__ out,
                                                            double* __restrict__ r2_trial) {
  __shared__ double red[256];
  double s = 0, k = 0, b0 = 0, b1 = 0;
  for (int64_t c = threadIdx.x; c < n_eval; c += 256) {
    if (!isnan(bps[c])) {
      s += bps[c];
      k += 1;
    }
    b0 += bad[2 * c];
    b1 += bad[2 * c + 1];
  }
  s = block_sum(s, red);
  k = block_sum(k, red);
  b0 = block_sum(b0, red);
  b1 = block_sum(b1, red);
  double rs = 0, rk = 0, nb = 0, se = 0, ae = 0;
  if (do_r2) {
    for (int64_t i = threadIdx.x; i < R; i += 256) {
      double m = 0;
      for (int64_t t = 0; t < T; ++t) {
        m += r2[i * T + t];
        nb += rowstat[3 * (i * T + t)];
        se += rowstat[3 * (i * T + t) + 1];
        ae += rowstat[3 * (i * T + t) + 2];
      }
      m /= (double)T;
      if (r2_trial) r2_trial[i] = m;
      if (!isnan(m)) {
        rs += m;
        rk += 1;
      }
    }
  }
  rs = block_sum(rs, red);
  rk = block_sum(rk, red);
  nb = block_sum(nb, red);
  se = block_sum(se, red);
  ae = block_sum(ae, red);
  if (threadIdx.x == 0) {
    const double nan = __builtin_nan("");
    const double total = (double)R * (double)T * (double)N;
    out[0] = k > 0 ? s / k : nan;
    out[1] = do_r2 && rk > 0 ? rs / rk : nan;
    out[2] = b0;
    out[3] = b1;
    out[4] = nb;
    out[5] = do_r2 && total > 0 ? se / total : nan;
    out[6] = do_r2 && total > 0 ? ae / total : nan;
  }
}

struct MetricsWs {
  int chunks;
  int64_t rows_per_chunk;
  size_t part, bps, bad, r2, rowstat, total;  // byte offsets
};
static MetricsWs metrics_ws(int64_t R, int64_t T, int64_t N) {
  MetricsWs w;
  const int64_t rows = R * T;
  const int64_t n_eval = R < N ? R : N;
  int64_t ch = cdiv(rows, 64);
  if (ch > kMaxChunks) ch = kMaxChunks;
  if (ch < 1) ch = 1;
  w.rows_per_chunk = cdiv(rows > 0 ? rows : 1, ch);
  w.chunks = (int)cdiv(rows > 0 ? rows : 1, w.rows_per_chunk);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  size_t off = 0;
  w.part = off;    off += al((size_t)w.chunks * kBpsStats * (n_eval > 0 ? n_eval : 1) * 8);
  w.bps = off;     off += al((size_t)(n_eval > 0 ? n_eval : 1) * 8);
  w.bad = off;     off += al((size_t)(n_eval > 0 ? n_eval : 1) * 16);
  w.r2 = off;      off += al((size_t)(rows > 0 ? rows : 1) * 8);
  w.rowstat = off; off += al((size_t)(rows > 0 ? rows : 1) * 24);
  w.total = off;
  return w;
}

}  // namespace vs

using namespace vs;

extern "C" size_t vs_spike_metrics_workspace_bytes(int64_t trials, int64_t T, int64_t N) {
  if (trials < 0 || T < 0 || N < 0) return 0;
  return metrics_ws(trials, T, N).total;
}

extern "C" int vs_spike_metrics(int64_t trials, int64_t T, int64_t N, const float* gt, const float* pred,
                                int32_t log_input, int64_t n_eval, int32_t want_r2, double* out,
                                double* bps_per_neuron, double* r2_per_trial, void* workspace, void* stream) {
  VS_REQUIRE(trials > 0 && T > 0 && N > 0, "vs_spike_metrics: empty input");
  VS_REQUIRE(gt && pred && out && workspace, "vs_spike_metrics: null pointer");
  VS_REQUIRE(n_eval >= 0 && n_eval <= N && n_eval <= trials, "vs_spike_metrics: n_eval must be <= min(trials, N)");
  VS_REQUIRE((((uintptr_t)workspace) & 15u) == 0, "vs_spike_metrics: workspace must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const MetricsWs w = metrics_ws(trials, T, N);
  char* ws = (char*)workspace;
  double* part = (double*)(ws + w.part);
  double* bps = bps_per_neuron ? bps_per_neuron : (double*)(ws + w.bps);
  double* bad = (double*)(ws + w.bad);
  double* r2 = (double*)(ws + w.r2);
  double* rowstat = (double*)(ws + w.rowstat);
  const int64_t rows = trials * T;
  if (n_eval > 0) {
    hipLaunchKernelGGL(bps_partial_kernel, dim3((unsigned)cdiv(n_eval, 256), (unsigned)w.chunks), dim3(256), 0, s, gt,
                       pred, rows, N, n_eval, (int)log_input, w.rows_per_chunk, part);
    hipLaunchKernelGGL(bps_neuron_kernel, dim3((unsigned)cdiv(n_eval, 256)), dim3(256), 0, s, (const double*)part,
                       w.chunks, n_eval, bps, bad);
  }
  if (want_r2)
    hipLaunchKernelGGL(r2_row_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, s, gt, pred, rows, N, (int)log_input,
                       r2, rowstat);
  hipLaunchKernelGGL(metrics_final_kernel, dim3(1), dim3(256), 0, s, (const double*)bps, (const double*)bad, n_eval,
                     (const double*)r2, (const double*)rowstat, trials, T, N, (int)want_r2, out, r2_per_trial);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
