// hg_knobs.hpp — tuning and test knobs of the library (hg_set_knob in
// include/horreum_gpu.h).  The library reads no environment variables: batch
// geometry overrides, A/B switches and test hooks are set explicitly through
// the C ABI, process-wide, and default to the measured best.
#pragma once
#include <stdint.h>

extern "C" int64_t hgk_knob(const char* name, int64_t dflt);
