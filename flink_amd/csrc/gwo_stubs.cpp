// temporary stubs (replaced as each engine lands)
#include "gwo_handle.h"
namespace gwo {
void Handle::comm_free() {}
gwo_status Handle::comm_exchange(const int64_t *, const int64_t *, const int64_t *, int64_t, const int64_t **, const int64_t **, const int64_t **, int64_t *) { return GWO_ERR_UNSUPPORTED; }
gwo_status Handle::comm_min_watermark(int64_t wm, int64_t *out) { *out = wm; return GWO_OK; }
}
extern "C" gwo_status gwo_comm_unique_id(uint8_t *) { return GWO_ERR_UNSUPPORTED; }
extern "C" gwo_status gwo_comm_init(gwo_handle *, const uint8_t *, int32_t, int32_t) { return GWO_ERR_UNSUPPORTED; }
