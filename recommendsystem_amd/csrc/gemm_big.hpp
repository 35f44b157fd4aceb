// The large-GEMM kernels of gemm_big.hip (the towers' Dense layers of >= 2^26 multiply-adds),
// called by the rs_dense_* entry points of dense.hip.
#pragma once
#include "common.hpp"

namespace rs_big {

enum { FORM_FWD = 0, FORM_DATA = 1, FORM_WEIGHT = 2 };
enum { EPI_FWD = 0, EPI_STORE = 1, EPI_PARTIAL = 2 };

struct Operand {
  const float* p;
  const float* y;    // a Z operand's Y (dZ = dY act'(Y), p = dY); nullptr: plain
  int64_t ld, ldy;
  int64_t X;         // output extent of this operand (rows of A / columns of B)
  int ones;          // WEIGHT A: output row X reads ones (the db row)
};

struct Args {
  Operand a, b;
  int64_t M, N, R;   // output M x N (M counts the db row), reduction length
  int64_t rchunk;    // reduction rows per split (set by the launcher)
  int act_z, epi, act;
  const float* bias;
  float* out;
  int64_t ldo;
  int accumulate;
  float* db;         // EPI_STORE: output row Mreal goes here
  int64_t Mreal;
  int64_t slab;      // EPI_PARTIAL: floats per split
  int tm, tn, gm;    // tile grid (set by the launcher)
  int xcd;           // re-index blocks so each XCD takes a contiguous tile range
};

struct Plan { int bm, bn, splits; int64_t rchunk; int stages; };

// the shapes that take these kernels (RS_GEMM_BIG=0 disables, RS_GEMM_BIG_MACS moves the bar)
bool wanted(int64_t m, int64_t n, int64_t k);
bool wanted_fwd(int64_t M, int64_t N, int64_t K);
Plan plan(int64_t M, int64_t N, int64_t R, bool allow_split, bool z);
// 0: launched; nonzero: not launched (unsupported tile / launch error)
int launch(hipStream_t s, int form, const Plan& p, const Args& g);
// the forward Y = act(X W + b), split-K through a library-owned partial slab when the tile grid
// alone cannot fill the chip (rs_dense_fwd has no workspace argument)
int fwd(hipStream_t s, const float* X, int64_t M, int64_t K, int64_t ldx, const float* W,
        const float* bias, int64_t N, int act, float* Y, int64_t ldy);

}  // namespace rs_big
