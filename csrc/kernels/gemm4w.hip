// Production instantiations of the 4-wave 256x256 GEMM (gemm4w.h): tile 34 (grouped tile
// order), 41 (deep weight ring), 45 (two-barrier K-tile, the prefill autotune's candidate).
#include "gemm4w.h"

template <int EPI>
static int dispatch_4w(int tile_cfg, DLI_GEMM_ARGS) {
  switch (tile_cfg) {
    // 256x256, one wave per SIMD, 128x128 wave tiles (gemm4w_kernel): 34 grouped order,
    // 41 = 34 with the deep weight ring (3 W stages, 160 KiB LDS)
    case 34: return launch_4w<EPI, 8>(DLI_GEMM_PASS);
    case 41: return launch_4w<EPI, 8 | 32>(DLI_GEMM_PASS);
    // 45 = 34 with the two-barrier schedule: the prefill autotune's 4-wave candidate
    case 45: return launch_4w<EPI, 8 | 4096>(DLI_GEMM_PASS);
    default: return DLI_NOT_MINE;
  }
}

int gemm_4w_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS) { DLI_EPI_SWITCH(dispatch_4w) }
int gemm_4w_set_slab_store(int mode) { return set_slab_store_tu(mode); }
