// Instantiates the ping-pong 8-wave GEMM tile menu (gemm_pp.h) for row-major A (CONV=0).
#include "gemm_pp.h"

GEMM_PP_TU_ENTRY(gemm_pp_c0_launch, 0)
