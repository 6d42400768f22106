// common.h -- error plumbing shared by the eegfx host sources (C++17, no torch types).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "eegfx.h"

namespace eegfx {

// Thread-local text behind eegfx_last_error().
void set_last_error(const std::string& msg);
const std::string& last_error();

// An error with a C-ABI status code.  Thrown inside the library, converted to a status at the
// extern "C" boundary (no exception ever crosses it).
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] inline void fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw Error(code, buf);
}

// Runs `f` and maps exceptions to status codes + last error text.
template <typename F>
int guarded(F&& f) {
  try {
    f();
    set_last_error("");
    return EEGFX_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("out of host memory");
    return EEGFX_ENOMEM;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return EEGFX_EINVAL;
  }
}

// ---- context accessors for the other host sources (api.cpp) -----------------------------------
int ctx_device(const eegfx_ctx* ctx);
void* ctx_stream(const eegfx_ctx* ctx);  // the context's hipStream_t

// ---- BrainVision reader (brainvision.cpp) ----------------------------------------------------
struct Header {
  eegfx_header_info info;
  std::vector<eegfx_channel_info> channels;
};
Header read_header(const std::string& vhdr_path);
std::vector<eegfx_marker> read_markers(const std::string& vmrk_path);
int64_t recording_frames(const Header& h, const std::string& eeg_path);
int sample_bytes(int32_t binary_format);
bool file_exists(const std::string& path);
// Reads the whole .eeg payload (n_frames * n_channels samples) into `dst`.
void read_file_bytes(const std::string& path, void* dst, int64_t nbytes);
// n_frames multiplexed frames of the recording (a VECTORIZED file is interleaved on the host).
void read_recording(const Header& h, const std::string& path, void* dst, int64_t n_frames);
// Java Integer.parseInt semantics (optional sign, ASCII digits, int32 range); false on failure.
bool java_parse_int(const std::string& s, int32_t* out);
// Java String.split(" ") semantics (trailing empty strings removed).
std::vector<std::string> java_split_space(const std::string& s);

}  // namespace eegfx
