// tile_order.hip -- the sort behind the sampling kernel's longest-tiles-first order (vdi_generate.hip,
// vdi_tile_len_kernel): one hipcub radix sort of (key, tile id) pairs per frame, descending.
#include <hipcub/hipcub.hpp>

#include "insitu_kernels.h"

namespace insitu {

hipError_t sort_tiles_desc(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                           const uint32_t* ids_in, uint32_t* ids_out, int n, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, keys_in, keys_out, ids_in, ids_out, n, 0,
                                                        32, s);
}

}  // namespace insitu
