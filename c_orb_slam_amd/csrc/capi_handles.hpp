// capi_handles.hpp -- the opaque C handles of include/orbslam_gpu.h (shared by the capi_*.cpp units).
#pragma once
#include "orb_extract.hpp"
#include "orb_match.hpp"

struct ORBextractor_t {
    orbgpu::Extractor* ex;
};

struct ORBmatcher_t {
    orbgpu::Matcher* m;
};
