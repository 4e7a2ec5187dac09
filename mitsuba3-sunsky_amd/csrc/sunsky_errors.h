// sunsky_errors.h -- error plumbing of the C ABI (include/sunsky_amd.h): C++
// exceptions never cross the boundary; every entry point returns a sunsky_status
// and leaves the message in a thread-local string (sunsky_last_error).
#pragma once
#include <hip/hip_runtime_api.h>

#include <stdexcept>
#include <string>

#include "sunsky_amd.h"

namespace sunsky {
namespace capi {

std::string& last_error();   // thread-local, sunsky_capi.cpp

inline int fail(int code, const std::string& msg) {
    last_error() = msg;
    return code;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct CommError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

// Runs f, mapping exceptions to status codes (the reference throws: logger.cpp:55-60).
template <typename F>
int guarded(F&& f) {
    try {
        f();
        return SUNSKY_OK;
    } catch (const HipError& e) {
        return fail(SUNSKY_ERROR_HIP, e.what());
    } catch (const CommError& e) {
        return fail(SUNSKY_ERROR_COMM, e.what());
    } catch (const std::invalid_argument& e) {
        return fail(SUNSKY_ERROR_INVALID_VALUE, e.what());
    } catch (const std::runtime_error& e) {
        std::string m = e.what();
        int code = (m.find("does not exist") != std::string::npos || m.find("cannot open") != std::string::npos)
                       ? SUNSKY_ERROR_FILE
                       : SUNSKY_ERROR_FORMAT;
        return fail(code, m);
    } catch (const std::exception& e) {
        return fail(SUNSKY_ERROR_INTERNAL, e.what());
    } catch (...) {
        return fail(SUNSKY_ERROR_INTERNAL, "unknown error");
    }
}

}  // namespace capi
}  // namespace sunsky
