// ctx.h — the device context shared by the batch API (host.cpp) and the streaming pipeline
// (pipeline.cpp).
#pragma once
#include <hip/hip_runtime.h>

struct pqgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // values kernels run here concurrently with k_levels (speculative mode)
};
