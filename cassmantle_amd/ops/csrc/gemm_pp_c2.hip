// Instantiates the ping-pong 8-wave GEMM tile menu (gemm_pp.h) for NHWC convs, Cin % 64 (CONV=2).
#include "gemm_pp.h"

GEMM_PP_TU_ENTRY(gemm_pp_c2_launch, 2)
