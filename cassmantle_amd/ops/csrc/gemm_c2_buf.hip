// Instantiates the MFMA GEMM / implicit-GEMM conv tile menu for A-operand mode CONV=2
// (0: row-major, 1: conv Cin%8, 2: conv Cin%64, 3: conv Cin%64 + fused 2x upsample), buffer-resource LDS-DMA.
// One translation unit per mode so the kernel library compiles in parallel (see gemm_impl.h).
#include "gemm_impl.h"

GEMM_TU_ENTRY(gemm_c2_buf_launch, 2, true)
