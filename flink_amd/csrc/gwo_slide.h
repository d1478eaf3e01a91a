// gwo_slide.h -- host state of sliding windows (gwo_slide.cpp: table panes; gwo_slog.cpp: logged panes).
#pragma once
#include <stdint.h>

#include <map>

#include "gwo_handle.h"

namespace gwo {

// A sliding window's entries restored from a per-window savepoint (gwo_import_heap_state: the heap backend keeps
// one accumulator per (key, window), WindowOperator.java:385-413, which cannot be split back into panes).  They
// stay per window and are combined into the window's rows when it fires (new records still go to panes), into its
// re-fire rows while it waits for its cleanup, and retire at its cleanup time.  Table layout: two hash tables --
// entries whose fire timer is pending (emitted at the fire) and entries whose window already fired (combined only
// into keys with new records in the window).  The sliding log keeps pending entries as a partial-accumulator
// segment (SlogState::rwins).
struct RestoredWindow {
    Table pend, done;             // base == nullptr: none
    uint64_t n_pend = 0, n_done = 0;
};

struct SlideState {
    bool ring = false;
    int count_word = -1;          // hidden per-entry count (ring): presence of a key in window J
    int t_idx = -1;               // aux_tables index of T
    bool j_set = false;
    __int128 J = 0;               // next window to fire
    unsigned long long *d_live = nullptr;
    unsigned long long h_live = 0;
    int64_t om = 0;               // floorMod(offset, slide): window j starts at j*slide + om
    std::map<long long, RestoredWindow> rwin;   // window index -> restored entries (table layout)
};

}  // namespace gwo
