// gso.hip — batched GSO split (worker/offload.cpp:46-216).  Kernel lands in
// the next commit; until then the entry point refuses loudly.
#include <hip/hip_runtime.h>

#include "wireglider_amd.h"

extern "C" int wg_gso_split(uint8_t *, const wg_gso_desc *, uint64_t, uint8_t *, wg_gso_result *, void *) {
    return WG_ERR_INVALID;
}
