// Device-side building blocks of the decode path (gfx950), shared by the standalone kernels and the
// fused attention block: decode_common.h (layout, prologues, epilogues, TP exchange), gemv_dev.h
// (the Q40 register-ring GEMV body), attn_dev.h (the decode attention task and split combine).
#pragma once

#include "decode_common.h"
#include "gemv_dev.h"
#include "attn_dev.h"
