// orb_extract.hpp -- host driver of the gfx950 ORB extractor (see orb_extract.hip).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>
#include <array>

#include "orb_common.hpp"
#include "octree.hpp"
#include "../../include/orbslam_gpu.h"

namespace orbgpu {

struct orb_kp_dev {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};
static_assert(sizeof(orb_kp_dev) == 28, "cv::KeyPoint layout");

struct CellDesc {          // one FAST cell ROI, ORBextractor.cc:794-829
    int r0, r1, c0, c1;    // ROI rows/cols in level interior coords
    int offx, offy;        // j*wCell, i*hCell (pt offset relative to minBorder)
    int pitch, cap, slot_off, level;
    long long lvl_off;     // byte offset of the padded level in an image slab
};

// Up to 2 x 2 neighbouring cells of one level (one k_fast_cells workgroup): their ROIs overlap by
// the 6-px FAST frame, so they tile one union ROI whose detection pixels are the cells' own,
// concatenated.  Cell k: bit 0 = right column, bit 1 = bottom row; cell[k] < 0 if absent.
struct CellGroup {
    int r0, c0, rows, cols;     // union ROI (level interior coords)
    int rsplit, csplit;         // detection rows of the top cells / columns of the left cells
    int pitch, pad;
    long long lvl_off;
    int cell[4], cap[4], slot_off[4];
    int xadd[4], yadd[4];       // union-ROI (col, row) + (xadd, yadd) = the cell's (offx, offy) + ROI (col, row)
};

struct BlurTile {
    long long off, boff;
    int pitch, bpitch, w, h, tx, ty;
};

// One destination tile of k_pyr_resize: padded-destination origin and the source
// rectangle it reads (interior rows [sr0, sr0+nsr), padded dword columns [sc0, sc0+4*nsw)).
constexpr int PT_W = 256, kPyrLdsMax = 48 * 1024;
struct PyrTile {
    int py0, px0, nrow, sr0, nsr, sc0, nsw, pad;
};

// k_pyr_chain: the levels [1, nlevels) of the pyramid in one launch, one workgroup per
// (row strip, image).  Per chained level: its padded geometry, the LDS buffer its computed rows
// live in (ping-pong between two buffers) and its resize tables (byte offsets into d_tabs_).
struct ChainLevel {
    long long off;
    int w, h, pitch, rp, lds, xofs, xal, yr, yb, nph;   // nph: threads per column group (row phases)
};
constexpr int kChainLdsMax = 64 * 1024;

// k_pyr_flow: the pyramid as one launch of dependent tasks; per level its padded geometry, its
// tasks and band counters, and (levels >= 1) its resize tables as byte offsets into d_tabs_
struct FlowLevel {
    long long off;          // padded level in the image slab
    int pitch, ph, w, h;
    int task0, ntiles;      // first task of the level (image 0); tasks per image
    int tile0;              // levels >= 1: the level's first PyrTile
    int band0, th, ncol;    // band counters: first slot, padded rows per band, tasks per band
    int xofs, xal, yr, yb;
};
struct FlowArgs {
    FlowLevel L[16];
    int nl, nbands;         // levels; band counters per image
};

struct LevelDev {
    long long off, boff;
    int pitch, bpitch;
    float scale, kp_size;
};
// every level's LevelDev by value, as a kernel argument (read with scalar loads)
constexpr int kMaxLevels = 16;
struct LevelArgs {
    LevelDev lv[kMaxLevels];
};

struct LevelHost {
    int w, h, pw, ph, pitch, bpitch;
    size_t off, boff;
};

class Extractor {
public:
    Extractor(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh);
    ~Extractor();
    int init_device(int maxW, int maxH, int maxBatch);
    // list != nullptr: B host images at list[b] (row stride step), staged as one block (imgs unused)
    int extract(const uint8_t* imgs, int B, int W, int H, int step, size_t img_stride, bool imgs_on_device,
                orb_kp* kps, uint8_t* desc, int cap, bool out_on_device, int* n_out,
                const uint8_t* const* list = nullptr);
    int get_level(int index, int level, uint8_t* dst, int dst_step, int* w, int* h);
    int get_blurred(int index, int level, uint8_t* dst, int dst_step, int* w, int* h);
    int timings(float* ms6);
    int corner_total(long long* total);   // FAST corners written by the last extract()
    hipStream_t stream() const { return stream_; }
    // recreate the stream with a CU mask leaving out one CU in every `one_in_n` (0: all CUs)
    int reserve_cus(int one_in_n);
    // launch on `with`'s stream (not owned; `with` must outlive this extractor)
    int share_stream(Extractor* with);
    int build_work(int B);
    // Device pyramid of the last extract() (mvImagePyramid with its 19-px border): image b's
    // padded level l starts at pyramid_base() + b * pyramid_image_bytes() + levels()[l].off.
    const uint8_t* pyramid_base() const { return (const uint8_t*)d_pyr_; }
    size_t pyramid_image_bytes() const { return img_bytes_; }
    const std::vector<LevelHost>& levels() const { return levels_; }
    int last_batch() const { return last_B_; }

    int nlevels() const { return nlevels_; }
    float scale_factor() const { return scaleFactor_; }
    const std::vector<float>& scale() const { return scale_; }
    const std::vector<float>& inv_scale() const { return invScale_; }
    const std::vector<float>& sigma2() const { return sigma2_; }
    const std::vector<float>& inv_sigma2() const { return invSigma2_; }
    const std::vector<int>& n_per_level() const { return nPerLevel_; }

private:
    static void gaussian_taps(int taps[7]);
    int setup_geometry(int W, int H);
    void release();

    int nfeatures_;
    double scaleFactorD_;
    float scaleFactor_;
    int nlevels_, iniTh_, minTh_;
    std::vector<float> scale_, invScale_, sigma2_, invSigma2_;
    std::vector<int> nPerLevel_, umax_;

    int maxW_ = 0, maxH_ = 0, maxB_ = 0;
    int geomW_ = -1, geomH_ = -1;
    std::vector<LevelHost> levels_;
    LevelArgs levelArgs_{};
    std::vector<CellDesc> cells_;
    std::vector<CellGroup> groups_;
    std::vector<int> level_cell_begin_;
    std::vector<BlurTile> tiles_;
    std::vector<PyrTile> ptiles_;
    std::vector<int> ptile_begin_, ptile_n_, plds_;   // per tile-height variant and level
    std::vector<int> ptile_th_;                       // rows per tile (band), per variant and level
    // k_pyr_flow (opt-in, ORBGPU_PYR_FLOW=1; default: a launch per level): band counters for
    // maxB_ images (zeroed before every launch) and the flow's dynamic LDS, per variant
    bool flow_ = false;
    int* d_flowcnt_ = nullptr;
    int flowBands_[2] = {0, 0}, flowLds_[2] = {0, 0};
    FlowArgs flow_args(int v, int B) const;
    // the chained pyramid (plan_chain): strips per image, dynamic LDS, device tables
    // [ChainLevel x (nlevels-1) | int4 strip ranges x K x (nlevels-1) | u16 padded rows]
    int plan_chain(const std::vector<std::vector<int>>& yr);
    bool chain_ = false;
    int chainK_ = 0, chainLds_ = 0, chainFrom_ = 0, chainSrcLds_ = 0, chainSrcRp_ = 0;
    std::vector<std::vector<int>> xofsAll_;     // every level's column map and taps (plan_chain)
    std::vector<std::vector<short>> xalAll_;
    size_t chainStripOff_ = 0, chainRowOff_ = 0;
    std::vector<uint8_t> chainTab_;
    void* d_chain_ = nullptr;
    void* d_cellslot_ = nullptr;   // slot offset of every cell (k_octree's compaction)
    std::vector<std::array<size_t, 4>> tab_off_;
    size_t img_bytes_ = 0, blur_bytes_ = 0, slots_per_image_ = 0;
    int packed_cap_ = 0, sel_cap_ = 0;
    int last_B_ = 0;

    hipStream_t stream_ = nullptr;
    bool ownStream_ = true;
    int lent_ = 0;   // extractors that launch on this one's stream (share_stream)
    hipEvent_t ev_[7] = {};
    // opt-in (ORBGPU_BLUR_SIDE=1): the blur runs on its own stream from the pyramid's end,
    // beside FAST / compaction / octree, and the descriptors wait for it
    hipStream_t side_ = nullptr;
    hipEvent_t evBlur_ = nullptr;
    // FAST of the large levels on side_ while the stream builds the small ones (opt-in,
    // ORBGPU_FAST_SPLIT=1)
    bool fastSplit_ = false;
    hipEvent_t evPyrA_ = nullptr, evFastA_ = nullptr;
    void *d_in_ = nullptr, *d_pyr_ = nullptr, *d_blur_ = nullptr, *d_slots_ = nullptr, *d_counts_ = nullptr;
    void *d_ptiles_ = nullptr;
    void *d_cells_ = nullptr, *d_tiles_ = nullptr, *d_lcb_ = nullptr, *d_packed_ = nullptr, *d_hdr_ = nullptr;
    void *d_sel_ = nullptr, *d_levels_ = nullptr, *d_tabs_ = nullptr, *d_kps_ = nullptr, *d_desc_ = nullptr;
    int* d_gtotal_ = nullptr;
    void* d_work_ = nullptr;   // k_fast_cells work order (build_work), for work_B_ images
    void* d_groups_ = nullptr;
    int work_B_ = -1, work_n_ = 0;
    int work_part_[2] = {0, 0};   // table entries of the levels < kFastSplitLevel, then of the rest
    bool d_gtotal_alias_ = false;
    size_t in_cap_ = 0, out_cap_ = 0;
    // host images go through this pinned block (a host memcpy, then an async DMA copy): the HIP
    // runtime's own path for pageable sources stalled an occasional call by several ms
    void* h_in_ = nullptr;
    size_t h_in_cap_ = 0;
    // device octree (octree.hip): per-job selections, per-image selected lists
    void *d_jobsel_ = nullptr, *d_jobcnt_ = nullptr, *d_octlv_ = nullptr, *d_gscr_ = nullptr, *d_nout_ = nullptr;
    int jcap_ = 0, selcap_ = 0;
    int* h_nout_ = nullptr;   // pinned: nout[maxB] + err

};

int debug_prof_extract(unsigned long long* out32);   // section timers of k_fast_cells (prof builds)

}  // namespace orbgpu
