// rt_sort.hip -- key/value radix sort for the ray queues (rocPRIM onesweep via hipCUB).
//
// The level-synchronous pipeline reorders each level's ray tasks and the frame's shadow
// rays by a spatial key (light or direction octant, then the Morton code of the ray
// origin) so that a wave's 64 rays walk nearly the same path through the culling
// hierarchy.  Order never changes a result: every task carries its parent slot and a
// shadow entry its node and light (rt_wavefront.hip).
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>

namespace rtdev {

// Sorts n (key, value) pairs on bits [0, end_bit) of the keys.  With tmp == nullptr only
// reports the scratch size in `bytes`.
hipError_t sort_pairs_u32(void* tmp, size_t& bytes, const uint32_t* keys_in, uint32_t* keys_out,
                          const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, int end_bit,
                          hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                              end_bit, stream);
}

}  // namespace rtdev
