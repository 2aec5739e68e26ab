// Epilogue parameter blocks of the implicit-GEMM convolutions (conv.hip); plain C layout shared
// with the torch bindings (conv_bindings.cpp).
#pragma once

namespace srl {
namespace conv {

struct EpiLNActP {  // z = acc, y = act(LN_c(z)), per-pixel mean/rstd
  float *z, *y, *mean, *rstd;
  const float *gamma, *beta;
  float eps;
  int act, M, y_nchw, lHW;
};
struct EpiLNBwdP {  // acc = dy; dz = LN/act backward; dgamma/dbeta += column sums
  const float *z, *mean, *rstd, *gamma, *beta;
  float *dz, *dgamma, *dbeta;
  float* part;    // [part_rows][2 * Nc] per-workgroup column sums (fixed-order reduce, no atomics); null -> atomics
  int part_rows;  // capacity of part in workgroups
  int defer;      // 1: leave part for a later conv_part_reduce_many (dgamma / dbeta unused)
  int act, M;
};
struct EpiPlainP {  // out = acc + bias + c0
  float* out;
  const float* bias;
  float c0;
  int M, Nreal, nchw, lHW;
};
struct ConvEpi {
  int mode;  // 0 LN_ACT, 1 LN_BWD, 2 PLAIN
  EpiLNActP ln;
  EpiLNBwdP lb;
  EpiPlainP pl;
};

}  // namespace conv
}  // namespace srl
