// The refine screen's descriptor-norm bound (refine.hip, SCREEN): max |D11h[pixel]|_2 as float bits (non-negative:
// ordered as unsigned; a NaN has the largest bits). The conversion blocks of the proj launch raise it by atomicMax,
// one atomic per block into slot (block % M3S_CMAX_SLOTS), the slots one 128-B line apart: a single word took the
// 4096 per-wave atomics of a 512x512 frame one after another (proj_occlusion 30 -> 64 us). prep zeroes the slots,
// the refine tile kernel max-reduces them.
#pragma once
#define M3S_CMAX_SLOTS 64
#define M3S_CMAX_STRIDE 32  // unsigned words between two slots (128 B)
