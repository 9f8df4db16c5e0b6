// gemm_dw.h — the token-reduction weight-gradient GEMM (gemm_dw.hip), used by vs_gemm.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "vspike.h"

namespace vs {

struct DwGrid {
  int tiles_m, tiles_n, splits, ksteps;  // ksteps: 64-token steps per split
};

struct DwPlan {
  bool valid, swap;  // swap: the kernel runs on (B, A) and stores C transposed
  int BM, BN;        // output tile: BM (64, 128, 192) rows of the narrow operand x BN (64, 128) columns
  int stages;        // LDS-DMA ring depth (3 or 4)
  DwGrid g;
  int64_t part_floats, sum_floats;
};

DwPlan plan_dw(int64_t M, int64_t N, int64_t K);
size_t dw_workspace_bytes(int64_t M, int64_t N, int64_t K);
int launch_dw(const vs_gemm_desc* d, hipStream_t s);

// skinny split-K (M <= 64, N <= 256, both operands K-contiguous, bf16 or f32): partials [splits][M][N] in the workspace
bool skinny_ok(const vs_gemm_desc* d);
size_t skinny_workspace_bytes(int32_t dtype, int64_t M, int64_t N, int64_t K);
int launch_skinny(const vs_gemm_desc* d, hipStream_t s, int* splits_out);

}  // namespace vs
