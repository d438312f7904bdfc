// capi_extract.cpp -- extern "C" ORBextractor_* entry points (include/orbslam_gpu.h).
// Each replaces a member of ORB_SLAM2::ORBextractor (reference include/ORBextractor.h).
#include <new>

#include "capi_handles.hpp"

extern "C" {

int orbgpu_device_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n > 0 ? 1 : 0;
}

const char* orbgpu_version(void) { return "c_orb_slam_amd 0.2 (gfx950)"; }
int orbgpu_abi_version(void) { return ORBGPU_ABI_VERSION; }

int ORBextractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                        int max_width, int max_height, int max_batch, ORBextractor_h* out) {
    if (!out || nfeatures < 0 || nlevels < 1 || nlevels > 15 || scaleFactor <= 1.0f || max_width <= 0 ||
        max_height <= 0 || max_batch <= 0 || max_batch > 2047)
        return ORB_E_INVALID;
    *out = nullptr;
    auto* ex = new (std::nothrow) orbgpu::Extractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST);
    if (!ex) return ORB_E_INVALID;
    int rc = ex->init_device(max_width, max_height, max_batch);
    if (rc) {
        delete ex;
        return rc == -4 ? ORB_E_NODEVICE : ORB_E_HIP;
    }
    *out = new ORBextractor_t{ex};
    return ORB_OK;
}

int ORBextractor_destroy(ORBextractor_h h) {
    if (!h) return ORB_E_INVALID;
    delete h->ex;
    delete h;
    return ORB_OK;
}

int ORBextractor_extract(ORBextractor_h h, const uint8_t* img, int width, int height, int step, orb_kp* kps,
                         uint8_t* desc, int capacity, int* n_out) {
    if (!h || !n_out) return ORB_E_INVALID;
    if (!img || width <= 0 || height <= 0) {  // ORBextractor.cc:1046-1047
        *n_out = 0;
        return ORB_OK;
    }
    return ORBextractor_extract_batch(h, img, 1, width, height, step, (size_t)step * height, 0, kps, desc, capacity,
                                      0, n_out);
}

int ORBextractor_extract_batch(ORBextractor_h h, const uint8_t* imgs, int batch, int width, int height, int step,
                               size_t img_stride, int imgs_on_device, orb_kp* kps, uint8_t* desc, int cap_per_image,
                               int outputs_on_device, int* n_out) {
    if (!h || !imgs || !kps || !desc || !n_out || batch <= 0 || step < width || cap_per_image < 0)
        return ORB_E_INVALID;
    int rc = h->ex->extract(imgs, batch, width, height, step, img_stride, imgs_on_device != 0, kps, desc,
                            cap_per_image, outputs_on_device != 0, n_out);
    if (rc == -3) return ORB_E_CAPACITY;
    if (rc == -2) return ORB_E_HIP;
    if (rc) return ORB_E_INVALID;
    return ORB_OK;
}

int ORBextractor_extract_images(ORBextractor_h h, const uint8_t* const* imgs, int batch, int width, int height,
                                int step, orb_kp* kps, uint8_t* desc, int cap_per_image, int outputs_on_device,
                                int* n_out) {
    if (!h || !imgs || !kps || !desc || !n_out || batch <= 0 || step < width || cap_per_image < 0 || height <= 0)
        return ORB_E_INVALID;
    for (int b = 0; b < batch; b++)
        if (!imgs[b]) return ORB_E_INVALID;
    int rc = h->ex->extract(nullptr, batch, width, height, step, (size_t)step * height, false, kps, desc,
                            cap_per_image, outputs_on_device != 0, n_out, imgs);
    if (rc == -3) return ORB_E_CAPACITY;
    if (rc == -2) return ORB_E_HIP;
    if (rc) return ORB_E_INVALID;
    return ORB_OK;
}

int ORBextractor_get_level(ORBextractor_h h, int index, int level, uint8_t* dst, int dst_step, int* w, int* h_) {
    if (!h || !w || !h_) return ORB_E_INVALID;
    int rc = h->ex->get_level(index, level, dst, dst_step, w, h_);
    return rc == 0 ? ORB_OK : (rc == -2 ? ORB_E_HIP : ORB_E_INVALID);
}

int ORBextractor_get_blurred_level(ORBextractor_h h, int index, int level, uint8_t* dst, int dst_step, int* w,
                                   int* h_) {
    if (!h || !w || !h_) return ORB_E_INVALID;
    int rc = h->ex->get_blurred(index, level, dst, dst_step, w, h_);
    return rc == 0 ? ORB_OK : (rc == -2 ? ORB_E_HIP : ORB_E_INVALID);
}

int ORBextractor_get_levels(ORBextractor_h h, int* nlevels, float* scaleFactor) {
    if (!h) return ORB_E_INVALID;
    if (nlevels) *nlevels = h->ex->nlevels();
    if (scaleFactor) *scaleFactor = h->ex->scale_factor();
    return ORB_OK;
}

int ORBextractor_get_scale_tables(ORBextractor_h h, float* scale, float* invScale, float* sigma2, float* invSigma2,
                                  int* nFeaturesPerLevel) {
    if (!h) return ORB_E_INVALID;
    const auto* ex = h->ex;
    for (int l = 0; l < ex->nlevels(); l++) {
        if (scale) scale[l] = ex->scale()[l];
        if (invScale) invScale[l] = ex->inv_scale()[l];
        if (sigma2) sigma2[l] = ex->sigma2()[l];
        if (invSigma2) invSigma2[l] = ex->inv_sigma2()[l];
        if (nFeaturesPerLevel) nFeaturesPerLevel[l] = ex->n_per_level()[l];
    }
    return ORB_OK;
}

void* ORBextractor_stream(ORBextractor_h h) { return h ? (void*)h->ex->stream() : nullptr; }

int ORBextractor_reserve_cus(ORBextractor_h h, int one_in_n) {
    if (!h || one_in_n < 0 || one_in_n == 1) return ORB_E_INVALID;
    const int r = h->ex->reserve_cus(one_in_n);
    return r == -4 ? ORB_E_NODEVICE : r == -1 ? ORB_E_INVALID : (r ? ORB_E_HIP : ORB_OK);
}

int ORBextractor_share_stream(ORBextractor_h h, ORBextractor_h with) {
    if (!h || !with) return ORB_E_INVALID;
    const int r = h->ex->share_stream(with->ex);
    return r == -4 ? ORB_E_NODEVICE : (r ? ORB_E_HIP : ORB_OK);
}

int ORBextractor_last_timings(ORBextractor_h h, float* ms6) {
    if (!h || !ms6) return ORB_E_INVALID;
    return h->ex->timings(ms6);
}

int ORBextractor_last_corner_count(ORBextractor_h h, long long* total) {
    if (!h || !total) return ORB_E_INVALID;
    return h->ex->corner_total(total) ? ORB_E_INVALID : ORB_OK;
}

}  // extern "C"
