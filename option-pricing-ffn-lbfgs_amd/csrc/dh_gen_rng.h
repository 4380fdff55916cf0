// dh_gen_rng.h -- the host part of the generator's device draw (dh_gen_device), shared between
// dh_gen_rng.cpp (host, g++) and dh_kernels.hip (the device side of the pipeline).
//
// The samples' positions in NumPy's legacy MT19937 stream depend on the data only through the
// polar method's acceptances, and the stream itself is one serial recurrence, so these two steps
// stay on one host: the twister (the MT19937 recurrence, publishing the key of every 64th
// generation) and the walk over the acceptance bitmaps (formed by a team of bit workers) that
// gives every sample its first double.  Everything else -- the words of the stream, the uniforms,
// the accepted pairs and their log / sqrt, the AR(1) blend and the spot walk -- runs on the device
// from those keys and positions (synthetic_generator.py:98-141).
#pragma once
#include <atomic>
#include <cstdint>

namespace dhgen {

constexpr int kMtWords = 624;
constexpr int kGensPerBlock = 64;     // generations per published key ("block")

struct Located {
    // ---- in: np.random.get_state()'s fields, the draw's size
    uint32_t key[kMtWords];
    int32_t pos = 0, has_gauss = 0;
    double gauss = 0.0;
    int64_t n = 0;                    // samples
    int n_opt = 0;                    // noise draws per sample (options)
    // ---- out buffers, caller-owned (locate_geometry sizes them):
    int64_t* t = nullptr;             // [n + 1]: sample i's first double (t[n]: after the last)
    int64_t* cs = nullptr;            // [n]: the value cached at sample i's start -- the first
                                      // double of the pair whose f x1 it is (>= 0), -1 the entry's
                                      // cached value, -2 none (has_gauss 0)
    uint32_t* keys = nullptr;         // [max_blocks][624]: the key of generation 64 b
    // ---- geometry (locate_geometry): word w >= 0 of the stream is key word (pos0 + w) % 624 of
    // generation (pos0 + w) / 624, generation 0 being the entry key (after a pending twist); the
    // walk never reads past double max_t
    int pos0 = 0;
    int64_t max_t = 0, max_blocks = 0;
    // ---- progress (release order): samples with t / cs written, blocks with keys written
    std::atomic<int64_t> located{0};
    std::atomic<int64_t> keys_ready{0};
    std::atomic<int> state{0};        // 0 running, 1 done, -1 past the stream bound
    // ---- out at the end: the state the reference's loop leaves (np.random.set_state's fields)
    uint32_t key_end[kMtWords];
    int32_t pos_end = 0, has_gauss_end = 0;
    double gauss_end = 0.0;
    double s_twister = 0.0, s_walk = 0.0;   // seconds from the start of locate_run
};

// pos0, max_t and max_blocks of L's draw (the caller sizes t, cs and keys from them)
void locate_geometry(Located& L);
// The twister, the bit workers and the walk on a team of threads, filling t, cs and keys as it
// goes; returns when the walk is done (L.state 1) or failed (-1).
void locate_run(Located& L);
// After locate_run: keys of blocks [L.keys_ready, blocks) that the twister stopped short of
// (twisted forward from the last published key).
void locate_extend_keys(Located& L, int64_t blocks);

}  // namespace dhgen
