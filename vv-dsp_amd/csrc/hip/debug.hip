// debug.hip -- the library's A/B switches ("knobs") and path counters.
//
// The launchers pick one kernel variant per call; the alternatives they can be
// switched to (older kernels kept for same-buffer A/B timing, and the static
// walks the dynamic ones are tested against) are selected through knobs, never
// through the environment at launch time:
//   * vvhip_debug_set(name, value) / vvhip_debug_clear(name) set or clear one
//     knob (atomics: safe against concurrent launches, unlike setenv/getenv);
//   * the environment is read ONCE, at the first knob query of the process, and
//     only when VVHIP_AB=1 is set (scripts/kbench.py's subprocess A/B runs), so
//     a stray VVHIP_* variable in a user's environment changes nothing.
// Path counters (STAT_*) count the launches of the paths tests must see taken
// (the dynamic walks, the fused signal -> mel kernel); vvhip_debug_get reads them.
#include "vvhip_internal.hpp"
#include "vv_dsp_hip.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace vvh {

namespace {
// knob names without the VVHIP_ prefix, in enum Knob order
constexpr const char* KNOB_NAMES[KNOB_COUNT] = {
    "STFT_CPS",      "STFT_RUN",     "STFT_DBS",     "POW_OLD",     "STFT_RING",   "STFT_DYN",
    "FS_VAR",        "FS_CHUNK_MB",  "FS_OLD",       "BLUE_UNFUSED", "C2C_MAX",    "STFT_SQ",     "MIX_VAR",
    "MIX_CHUNK_MB",  "MIX_R2C_FULL", "FIR_OLD",      "FIR_DYN",     "FIR_DIRECT_LDS", "FIR_BLOCK",
    "HOST_CHUNK_MB", "NO_MIXED",     "REAL_PROMOTE", "ISTFT_OLD",   "MEL_FUSED",   "CZT_UNFUSED",
    "CEPS_UNFUSED",  "FIR_R32",      "DIST_SLAB_KB", "POW_R32", "MAG_R32",     "MEL_R32", "C2C_TPW", "C2C_ONE", "REAL_TPW", "ANA_TPW", "MIX_TPW", "C2C_SMALL", "DCT_SMALL", "HIL_SMALL", "REAL_SMALL", "R2C_SMALL", "STFT_STAGE", "STFT_ONE", "MFCC_WIN",
};
constexpr const char* STAT_NAMES[STAT_COUNT] = {
    "STAT_STFT_DYN", "STAT_FIR_DYN", "STAT_FIR_STATIC", "STAT_MEL_FUSED", "STAT_MEL_SPLIT", "STAT_FIR_R32", "STAT_POW_R32", "STAT_MAG_R32", "STAT_MEL_R32",
};
constexpr long long UNSET = -1;

std::atomic<long long> g_knob[KNOB_COUNT];
std::atomic<long long> g_stat[STAT_COUNT];
std::once_flag g_env_once;

const char* env(const char* name) { return std::getenv(name); }   // the library's only read of VVHIP_* variables

void load_env() {
    for (auto& k : g_knob) k.store(UNSET, std::memory_order_relaxed);
    const char* ab = env("VVHIP_AB");
    if (!(ab && ab[0] == '1')) return;
    char buf[64];
    for (int i = 0; i < KNOB_COUNT; ++i) {
        std::snprintf(buf, sizeof buf, "VVHIP_%s", KNOB_NAMES[i]);
        const char* v = env(buf);
        if (v && *v) g_knob[i].store(std::atoll(v), std::memory_order_relaxed);
    }
}

void init() { std::call_once(g_env_once, load_env); }

// "STFT_DYN" or "VVHIP_STFT_DYN" -> knob index; "STAT_..." -> STAT_COUNT + stat index; -1 unknown
int lookup(const char* name) {
    if (!name) return -1;
    if (std::strncmp(name, "VVHIP_", 6) == 0) name += 6;
    for (int i = 0; i < KNOB_COUNT; ++i)
        if (std::strcmp(name, KNOB_NAMES[i]) == 0) return i;
    for (int i = 0; i < STAT_COUNT; ++i)
        if (std::strcmp(name, STAT_NAMES[i]) == 0) return KNOB_COUNT + i;
    return -1;
}
}  // namespace

long long knob(Knob k, long long dflt) {
    init();
    const long long v = g_knob[k].load(std::memory_order_relaxed);
    return v == UNSET ? dflt : v;
}

void stat_inc(Stat s) { g_stat[s].fetch_add(1, std::memory_order_relaxed); }

}  // namespace vvh

extern "C" {

__attribute__((visibility("default"))) int vvhip_debug_set(const char* name, long long value) {
    vvh::init();
    const int i = vvh::lookup(name);
    if (i < 0 || i >= vvh::KNOB_COUNT || value < 0) return -1;
    vvh::g_knob[i].store(value, std::memory_order_relaxed);
    return 0;
}

__attribute__((visibility("default"))) int vvhip_debug_clear(const char* name) {
    vvh::init();
    if (!name) {   // every knob back to the default path, every path counter to 0
        for (auto& k : vvh::g_knob) k.store(vvh::UNSET, std::memory_order_relaxed);
        for (auto& c : vvh::g_stat) c.store(0, std::memory_order_relaxed);
        return 0;
    }
    const int i = vvh::lookup(name);
    if (i < 0) return -1;
    if (i < vvh::KNOB_COUNT) vvh::g_knob[i].store(vvh::UNSET, std::memory_order_relaxed);
    else vvh::g_stat[i - vvh::KNOB_COUNT].store(0, std::memory_order_relaxed);
    return 0;
}

__attribute__((visibility("default"))) long long vvhip_debug_get(const char* name) {
    vvh::init();
    const int i = vvh::lookup(name);
    if (i < 0) return -2;
    if (i < vvh::KNOB_COUNT) return vvh::g_knob[i].load(std::memory_order_relaxed);
    return vvh::g_stat[i - vvh::KNOB_COUNT].load(std::memory_order_relaxed);
}

}  // extern "C"
