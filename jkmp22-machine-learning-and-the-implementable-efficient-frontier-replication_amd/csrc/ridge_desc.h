// Cell descriptor shared by the ridge-grid kernels (ridge.hip: tridiagonal path,
// ridge_band.hip: band path).  Layout mirrors ops/ridge.py::CELL_DTYPE.
#pragma once
#include <stdint.h>

struct RidgeCellDesc {
  int64_t src;      // offset (doubles) of the running-sum matrix S_D for this cell
  int64_t rsrc;     // offset of the running-sum vector S_r
  int64_t work;     // offset of this cell's workspace
  int64_t out;      // offset of beta output [L][ldo]
  int n;            // p + 1
  double scale;     // 1 / T  (the reference divides both sums by n months)
};
