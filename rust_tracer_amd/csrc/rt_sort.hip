// rt_sort.hip -- key/value radix sort for the ray queues (rocPRIM onesweep).
//
// The level-synchronous pipeline reorders each level's ray tasks and the frame's shadow
// rays by a spatial key (light or direction octant, then the Morton code of the ray
// origin) so that a wave's 64 rays walk nearly the same path through the culling
// hierarchy.  Order never changes a result: every task carries its parent slot and a
// shadow entry its node and light (rt_wavefront.hip).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

namespace rtdev {

// Sorts n (key, value) pairs on bits [0, end_bit) of the keys.  With tmp == nullptr only
// reports the scratch size in `bytes`.
// Onesweep at every size: rocPRIM's default switches to a merge sort below 1M items,
// which is 3-4x slower on these 18-20 bit keys (every per-level task sort is < 1M).
using onesweep_only = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                 rocprim::default_config, 0>;

hipError_t sort_pairs_u32(void* tmp, size_t& bytes, const uint32_t* keys_in, uint32_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, int end_bit,
                          hipStream_t stream) {
    return rocprim::radix_sort_pairs<onesweep_only>(tmp, bytes, keys_in, keys_out, vals_in, vals_out, n, 0,
                                                    (unsigned int)end_bit, stream);
}

}  // namespace rtdev
