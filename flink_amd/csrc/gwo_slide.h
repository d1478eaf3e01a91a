// gwo_slide.h -- host state of sliding windows (gwo_slide.cpp: table panes; gwo_slog.cpp: logged panes).
#pragma once
#include <stdint.h>

namespace gwo {

struct SlideState {
    bool ring = false;
    int count_word = -1;          // hidden per-entry count (ring): presence of a key in window J
    int t_idx = -1;               // aux_tables index of T
    bool j_set = false;
    __int128 J = 0;               // next window to fire
    unsigned long long *d_live = nullptr;
    unsigned long long h_live = 0;
    int64_t om = 0;               // floorMod(offset, slide): window j starts at j*slide + om
};

}  // namespace gwo
