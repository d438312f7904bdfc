// stereo.hpp -- gfx950 Frame::ComputeStereoMatches (see stereo.hip).  Reference src/Frame.cc:466-640.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "orb_common.hpp"
#include "orb_extract.hpp"

namespace orbgpu {

constexpr int kStereoMaxKeys = 4096;
constexpr int kStereoMaxLevels = 16;
constexpr int kStereoMaxRows = 4096;   // mvImagePyramid[0].rows (the row table lives in LDS)

struct StereoLevel {   // padded level l of one image slab: (0,0) of the unpadded level at +19 rows/cols
    long long off;
    int pitch, w, h;
};

struct StereoParams {
    StereoLevel lv[kStereoMaxLevels];
    float scale[kStereoMaxLevels], invScale[kStereoMaxLevels];
    float mbf, mb;
    int rows0;         // mvImagePyramid[0].rows
};

// one stereo pair
struct StereoDev {
    int NL, NR;
    const orb_kp_dev* kL;   // mvKeys (left)
    const uint8_t* dL;      // mDescriptors
    const orb_kp_dev* kR;   // mvKeysRight
    const uint8_t* dR;      // mDescriptorsRight
    const uint8_t* pyrL;    // left extractor pyramid slab of this image
    const uint8_t* pyrR;
    float* uRight;          // out: mvuRight (NL)
    float* depth;           // out: mvDepth (NL)
    int* sad;               // scratch (NL): best SAD or -1
    int* kept;              // out: stereo matches after the median filter
    int* rowStart;          // scratch (rows0 + 1): vRowIndices as CSR (Frame.cc:476-493)
    int2* rowIdx;           // scratch (NR * band rows): (uR bits, iR | octave << 24) per entry
};

class Matcher;
// tm (optional): the matcher whose timing events / counters record the launches (its stream is s)
int stereo_launch(const StereoDev* d_probs, int nprob, int maxNL, const StereoParams& P, hipStream_t s,
                  Matcher* tm = nullptr);

// Frame::UnprojectStereo over a batch of frames (Frame.cc:666-680)
struct UnprojDev {
    int N;
    const orb_kp_dev* keys;
    const float* depth;
    const float* Twc;
    float fx, fy, cx, cy, invfx, invfy;
    float* x3D;
    int* mp;
    // new map points (MapPoint_CreateStereo): row ids from mp_base, UpdateNormalAndDepth outputs
    int mp_base;
    float* normal;      // null: UnprojectStereo only
    float* maxDist;
    float* minDist;
    const float* scale;
    int nlevels;
};

// Tracking's bookkeeping between TrackWithMotionModel's PoseOptimization and SearchLocalPoints
struct LocalPrepDev {
    int N;
    int* curMP;
    const uint8_t* outlier;
    int n;
    const int* row;
    uint8_t* skip;
};
int local_prep_batch(const LocalPrepDev* d_probs, int count, hipStream_t s);
constexpr int kUnprojPerLaunch = 56;   // frames per launch, passed by value (kernel-argument space)
// enqueue on `s` (no staging buffer: the frames are kernel arguments)
int unproject_batch(const UnprojDev* probs, int count, hipStream_t s);

// Frame::UndistortKeyPoints over a batch of frames (Frame.cc:404-430): cv::undistortPoints
// (OpenCV 3.2 cvUndistortPoints, R = I, P = K) on every keypoint; the rest of the KeyPoint is
// copied.  has_dist = 0 (mDistCoef.at<float>(0) == 0) copies mvKeys.
struct UndistDev {
    int N, has_dist;
    const orb_kp_dev* keys;
    orb_kp_dev* keysUn;
    double A[9];   // mK as double (cvConvert)
    double k[8];   // k1 k2 p1 p2 k3 k4 k5 k6 as double, zero-filled
};
constexpr int kUndistPerLaunch = 24;   // frames per launch, passed by value
int undistort_batch(const UndistDev* probs, int count, hipStream_t s);

}  // namespace orbgpu
