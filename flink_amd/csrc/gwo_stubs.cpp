// temporary stubs (replaced as each engine lands)
#include "gwo_handle.h"
namespace gwo {
gwo_status Handle::slide_init() { return fail(GWO_ERR_UNSUPPORTED, "sliding not built yet"); }
void Handle::slide_free() {}
gwo_status Handle::fire_sliding(int64_t) { return GWO_ERR_UNSUPPORTED; }
gwo_status Handle::session_init() { return fail(GWO_ERR_UNSUPPORTED, "sessions not built yet"); }
void Handle::session_free() {}
gwo_status Handle::insert_session(const int64_t *, const int64_t *, const int64_t *, int64_t) { return GWO_ERR_UNSUPPORTED; }
gwo_status Handle::fire_session(int64_t) { return GWO_ERR_UNSUPPORTED; }
gwo_status Handle::session_state_size(int64_t *) { return GWO_ERR_UNSUPPORTED; }
void Handle::comm_free() {}
gwo_status Handle::comm_exchange(const int64_t *, const int64_t *, const int64_t *, int64_t, const int64_t **, const int64_t **, const int64_t **, int64_t *) { return GWO_ERR_UNSUPPORTED; }
gwo_status Handle::comm_min_watermark(int64_t wm, int64_t *out) { *out = wm; return GWO_OK; }
}
extern "C" gwo_status gwo_comm_unique_id(uint8_t *) { return GWO_ERR_UNSUPPORTED; }
extern "C" gwo_status gwo_comm_init(gwo_handle *, const uint8_t *, int32_t, int32_t) { return GWO_ERR_UNSUPPORTED; }
