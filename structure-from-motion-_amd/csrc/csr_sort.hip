// The camera-major permutation of a BA problem's observations on the device
// (round 5, sfm_ba_create): a stable LSD radix sort of the camera indices
// (rocPRIM, only the bits the camera count needs) with the observation index
// as the value, so each camera's observations stay in point order -- the
// host counting sort's cam_obs, bit for bit.  Kept in its own translation
// unit: rocPRIM's templates are heavy and ba.hip is big already.
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "sfm_common.hpp"

namespace sfm {

// temp_bytes == 0 on entry: only the size is returned (rocPRIM's convention)
int cam_major_sort(void *temp, size_t &temp_bytes, const int32_t *cam, uint32_t *keys_out, int32_t *perm_out,
                   int64_t no, int32_t nc, hipStream_t s) {
    int bits = 1;
    while (bits < 31 && (1 << bits) < nc) ++bits;
    const hipError_t e = rocprim::radix_sort_pairs(temp, temp_bytes, reinterpret_cast<const uint32_t *>(cam), keys_out,
                                                   rocprim::counting_iterator<int32_t>(0), perm_out, (size_t)no, 0,
                                                   bits, s);
    return e == hipSuccess ? 0 : SFM_ERR_HIP;
}

}  // namespace sfm
