// Instantiates the halo-staged 3x3 convolution (gemm_halo.h): tile configs 24 (256x160) and
// 25 (128x160), chosen only from the measured tuning table or when forced.
#include "gemm_halo.h"

bool gemm_halo_ok(const GemmArgs& p, int cfg) { return halo_ok(p, halo_bm(cfg - 24), halo_bn(cfg - 24)); }
