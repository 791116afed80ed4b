// temporary: tracker entry points (replaced by tracker.hip)
#include "ctx.h"
extern "C" {
int erp_klt_track(vio_ctx*, const uint8_t*, const uint8_t*, int, int, int, const float*, int, float*, uint8_t*, float*,
                  const erp_klt_params*) { return VIO_ENOSYS; }
int erp_gftt(vio_ctx*, const uint8_t*, const uint8_t*, int, int, int, int, double, double, float*, int*) { return VIO_ENOSYS; }
int erp_rot_ransac(vio_ctx*, const float*, const float*, int, int, int, const int32_t*, int, float, uint8_t*, int*) { return VIO_ENOSYS; }
int erp_tracker_create(vio_ctx*, int, int, int, int, erp_tracker**) { return VIO_ENOSYS; }
int erp_tracker_upload(erp_tracker*, int, const uint8_t*, int) { return VIO_ENOSYS; }
int erp_tracker_set_points(erp_tracker*, const float*, int, const int32_t*, int) { return VIO_ENOSYS; }
int erp_tracker_run(erp_tracker*, const erp_klt_params*, const erp_tracker_params*) { return VIO_ENOSYS; }
int erp_tracker_sync(erp_tracker*) { return VIO_ENOSYS; }
int erp_tracker_download(erp_tracker*, float*, uint8_t*, uint8_t*, float*, int*) { return VIO_ENOSYS; }
int erp_tracker_kernel_ms(erp_tracker*, double*, double*, double*, double*) { return VIO_ENOSYS; }
void erp_tracker_destroy(erp_tracker*) {}
}
