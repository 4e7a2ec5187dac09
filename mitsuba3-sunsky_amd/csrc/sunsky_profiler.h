// sunsky_profiler.h -- profiler ranges around the C-ABI batch entry points, the
// counterpart of the reference's MI_MASKED_FUNCTION(ProfilerPhase::...) scopes
// (sunsky.cpp:304 eval, :358 sample_ray, :402 sample_direction, :444
// pdf_direction, :454 eval_direction; phase names from
// include/mitsuba/core/profiler.h).  Each scope is a roctx range
// "<phase>:<entry point>" on the calling thread, so `rocprofv3 --marker-trace`
// shows the host-side span of every call (argument checks, staging, launches)
// next to the kernels it enqueued.  With no tool attached a push/pop pair costs a
// few tens of nanoseconds; SUNSKY_AMD_ROCTX=0 turns the ranges off.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>
#include <cstring>

namespace sunsky {

inline bool roctx_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SUNSKY_AMD_ROCTX");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}

class ProfilerPhase {
public:
    explicit ProfilerPhase(const char* name) : on_(roctx_enabled()) {
        if (on_) roctxRangePushA(name);
    }
    ~ProfilerPhase() {
        if (on_) roctxRangePop();
    }
    ProfilerPhase(const ProfilerPhase&) = delete;
    ProfilerPhase& operator=(const ProfilerPhase&) = delete;

private:
    bool on_;
};

}  // namespace sunsky

#define SUNSKY_PHASE(phase, entry) ::sunsky::ProfilerPhase sunsky_profiler_phase_(phase ":" entry)
