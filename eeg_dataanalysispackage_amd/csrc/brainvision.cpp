// brainvision.cpp -- native BrainVision reader and marker planner (host side of the hot path).
//
// Replaces the un-vendored eegloader-hdfs 2.4 (cz.zcu.kiv.signal.*, pom.xml:84-88) calls made by
// OffLineDataProvider.processEEGFiles:
//   getChannelInfo(vhdr)        OffLineDataProvider.java:167-168
//   readMarkerList(vmrk)        OffLineDataProvider.java:196
// and restates the per-marker selection of OffLineDataProvider.java:200-265 (stimulus index,
// out-of-range skip, target label, class balance) as eegfx_plan_markers.  The binary decode of
// readBinaryData (:185-188) is fused into the device kernels (kernels.hip); this file only
// moves the raw bytes.
#include <sys/stat.h>

#include <cctype>
#include <cerrno>
#include <climits>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "common.h"

namespace eegfx {

namespace {
thread_local std::string g_last_error;

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\t' || s[b] == '\r' || s[b] == '\n')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r' || s[e - 1] == '\n')) --e;
  return s.substr(b, e - b);
}

std::string lower(std::string s) {
  for (auto& ch : s) ch = (char)std::tolower((unsigned char)ch);
  return s;
}

// BrainVision escapes commas inside a field as "\1".
std::string unescape(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 1 < s.size() && s[i + 1] == '1') {
      out.push_back(',');
      ++i;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

std::vector<std::string> split_commas(const std::string& s) {
  std::vector<std::string> parts;
  std::string cur;
  for (char ch : s) {
    if (ch == ',') {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  parts.push_back(cur);
  return parts;
}

void copy_field(char* dst, size_t cap, const std::string& s) {
  size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
  memcpy(dst, s.data(), n);
  dst[n] = 0;
}

// Reads a text file into lines (handles \n, \r\n and \r like BufferedReader.readLine).
std::vector<std::string> read_lines(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) fail(EEGFX_EIO, "cannot open %s", path.c_str());
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  std::vector<std::string> lines;
  std::string cur;
  for (size_t i = 0; i < text.size(); ++i) {
    char ch = text[i];
    if (ch == '\n' || ch == '\r') {
      lines.push_back(cur);
      cur.clear();
      if (ch == '\r' && i + 1 < text.size() && text[i + 1] == '\n') ++i;
    } else {
      cur.push_back(ch);
    }
  }
  if (!cur.empty()) lines.push_back(cur);
  return lines;
}

bool parse_int64(const std::string& s, int64_t* out) {
  std::string t = trim(s);
  if (t.empty()) return false;
  char* end = nullptr;
  errno = 0;
  long long v = strtoll(t.c_str(), &end, 10);
  if (errno != 0 || *end != 0) return false;
  *out = v;
  return true;
}

bool parse_double(const std::string& s, double* out) {
  std::string t = trim(s);
  if (t.empty()) return false;
  char* end = nullptr;
  double v = strtod(t.c_str(), &end);
  if (*end != 0) return false;
  *out = v;
  return true;
}
}  // namespace

void set_last_error(const std::string& msg) { g_last_error = msg; }
const std::string& last_error() { return g_last_error; }

bool java_parse_int(const std::string& s, int32_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  int64_t v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
    if (v > (int64_t)INT_MAX + 1) return false;
  }
  if (neg) v = -v;
  if (v < INT_MIN || v > INT_MAX) return false;
  *out = (int32_t)v;
  return true;
}

std::vector<std::string> java_split_space(const std::string& s) {
  std::vector<std::string> parts;
  std::string cur;
  for (char ch : s) {
    if (ch == ' ') {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  parts.push_back(cur);
  while (!parts.empty() && parts.back().empty()) parts.pop_back();  // String.split drops trailing ""
  if (parts.empty() && !s.empty()) return parts;  // " " -> []
  if (s.empty()) return {""};                     // "".split(" ") -> [""]
  return parts;
}

bool file_exists(const std::string& path) {
  struct stat st;
  return stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

int sample_bytes(int32_t binary_format) { return binary_format == EEGFX_IEEE_FLOAT_32 ? 4 : 2; }

Header read_header(const std::string& vhdr_path) {
  Header h;
  memset(&h.info, 0, sizeof(h.info));
  h.info.binary_format = EEGFX_INT_16;
  h.info.multiplexed = 1;
  std::string section;
  bool have_nch = false;
  for (const std::string& raw : read_lines(vhdr_path)) {
    std::string line = trim(raw);
    if (line.empty() || line[0] == ';') continue;
    if (line[0] == '[') {
      section = lower(line);
      if (section == "[comment]") break;  // free text follows
      continue;
    }
    size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::string key = trim(line.substr(0, eq)), val = line.substr(eq + 1);
    if (section == "[common infos]") {
      if (key == "NumberOfChannels") {
        int64_t v;
        if (!parse_int64(val, &v) || v <= 0 || v > 65536)
          fail(EEGFX_EFORMAT, "%s: bad NumberOfChannels '%s'", vhdr_path.c_str(), val.c_str());
        h.info.n_channels = (int32_t)v;
        have_nch = true;
      } else if (key == "DataFile") {
        copy_field(h.info.data_file, sizeof(h.info.data_file), trim(val));
      } else if (key == "MarkerFile") {
        copy_field(h.info.marker_file, sizeof(h.info.marker_file), trim(val));
      } else if (key == "DataOrientation") {
        std::string v = trim(val);
        if (v == "MULTIPLEXED") h.info.multiplexed = 1;
        else if (v == "VECTORIZED") h.info.multiplexed = 0;
        else fail(EEGFX_EFORMAT, "%s: unknown DataOrientation '%s'", vhdr_path.c_str(), v.c_str());
      } else if (key == "SamplingInterval") {
        double v;
        if (parse_double(val, &v)) h.info.sampling_interval_us = v;
      } else if (key == "DataFormat") {
        if (trim(val) != "BINARY")
          fail(EEGFX_ENOTSUP, "%s: DataFormat '%s' (only BINARY)", vhdr_path.c_str(), val.c_str());
      }
    } else if (section == "[binary infos]") {
      if (key == "BinaryFormat") {
        std::string v = trim(val);
        if (v == "INT_16") h.info.binary_format = EEGFX_INT_16;
        else if (v == "IEEE_FLOAT_32") h.info.binary_format = EEGFX_IEEE_FLOAT_32;
        else fail(EEGFX_ENOTSUP, "%s: BinaryFormat '%s'", vhdr_path.c_str(), v.c_str());
      }
    } else if (section == "[channel infos]") {
      if (key.size() > 2 && key[0] == 'C' && key[1] == 'h') {
        int64_t num;
        if (!parse_int64(key.substr(2), &num) || num <= 0)
          fail(EEGFX_EFORMAT, "%s: bad channel key '%s'", vhdr_path.c_str(), key.c_str());
        std::vector<std::string> f = split_commas(val);
        eegfx_channel_info ci;
        memset(&ci, 0, sizeof(ci));
        ci.number = (int32_t)num;
        copy_field(ci.name, sizeof(ci.name), unescape(f.size() > 0 ? f[0] : ""));
        copy_field(ci.reference, sizeof(ci.reference), unescape(f.size() > 1 ? f[1] : ""));
        ci.resolution = 1.0;
        if (f.size() > 2 && !trim(f[2]).empty() && !parse_double(f[2], &ci.resolution))
          fail(EEGFX_EFORMAT, "%s: bad resolution '%s'", vhdr_path.c_str(), f[2].c_str());
        copy_field(ci.unit, sizeof(ci.unit), f.size() > 3 ? f[3] : "");
        h.channels.push_back(ci);
      }
    }
  }
  if (!have_nch) fail(EEGFX_EFORMAT, "%s: missing NumberOfChannels", vhdr_path.c_str());
  return h;
}

std::vector<eegfx_marker> read_markers(const std::string& vmrk_path) {
  std::vector<eegfx_marker> out;
  std::string section;
  for (const std::string& raw : read_lines(vmrk_path)) {
    std::string line = trim(raw);
    if (line.empty() || line[0] == ';') continue;
    if (line[0] == '[') {
      section = lower(line);
      continue;
    }
    if (section != "[marker infos]") continue;
    size_t eq = line.find('=');
    if (eq == std::string::npos || line.compare(0, 2, "Mk") != 0) continue;
    eegfx_marker m;
    memset(&m, 0, sizeof(m));
    int64_t num;
    if (!parse_int64(line.substr(2, eq - 2), &num))
      fail(EEGFX_EFORMAT, "%s: bad marker key '%s'", vmrk_path.c_str(), line.c_str());
    m.number = (int32_t)num;
    std::vector<std::string> f = split_commas(line.substr(eq + 1));
    if (f.size() < 3) fail(EEGFX_EFORMAT, "%s: short marker '%s'", vmrk_path.c_str(), line.c_str());
    copy_field(m.type, sizeof(m.type), unescape(f[0]));
    const std::string desc = unescape(f[1]);
    copy_field(m.description, sizeof(m.description), desc);
    if (!parse_int64(f[2], &m.position))
      fail(EEGFX_EFORMAT, "%s: bad marker position '%s'", vmrk_path.c_str(), f[2].c_str());
    m.size = 1;
    if (f.size() > 3) parse_int64(f[3], &m.size);
    int64_t ch = 0;
    if (f.size() > 4 && parse_int64(f[4], &ch)) m.channel = (int32_t)ch;
    // OffLineDataProvider.java:207-214: marker.getStimulus().replaceAll("[\\D]", "") then
    // Integer.parseInt(...) - 1, or -1 when no digit is left.
    std::string digits;
    for (char c : desc)
      if (c >= '0' && c <= '9') digits.push_back(c);
    if (digits.empty()) {
      m.stimulus_index = -1;
    } else {
      int32_t v;
      // NumberFormatException on int overflow: flagged, raised by the planner in order.
      m.stimulus_index = java_parse_int(digits, &v) ? v - 1 : INT32_MIN;
    }
    out.push_back(m);
  }
  return out;
}

int64_t recording_frames(const Header& h, const std::string& eeg_path) {
  struct stat st;
  if (stat(eeg_path.c_str(), &st) != 0) fail(EEGFX_EIO, "cannot stat %s", eeg_path.c_str());
  const int64_t frame = (int64_t)h.info.n_channels * sample_bytes(h.info.binary_format);
  return (int64_t)st.st_size / frame;
}

void read_file_bytes(const std::string& path, void* dst, int64_t nbytes) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) fail(EEGFX_EIO, "cannot open %s", path.c_str());
  int64_t got = 0;
  char* p = (char*)dst;
  while (got < nbytes) {
    size_t r = fread(p + got, 1, (size_t)(nbytes - got), f);
    if (r == 0) break;
    got += (int64_t)r;
  }
  fclose(f);
  if (got != nbytes) fail(EEGFX_EIO, "short read on %s (%lld of %lld bytes)", path.c_str(),
                          (long long)got, (long long)nbytes);
}

// The recording as multiplexed frames ([n_frames][n_channels] samples), whatever the file's
// DataOrientation.  A VECTORIZED file stores channel after channel ([n_channels][n_frames]); it is
// interleaved here, on the host while it is read, so every kernel sees one layout.  eegloader's
// readBinaryData demultiplexes either orientation to per-channel arrays (OffLineDataProvider.java:
// 185-188); parity unpinned for VECTORIZED -- no file of the reference's test data uses it.
void read_recording(const Header& h, const std::string& path, void* dst, int64_t n_frames) {
  const int64_t sb = sample_bytes(h.info.binary_format), nc = h.info.n_channels;
  const int64_t nbytes = n_frames * nc * sb;
  if (h.info.multiplexed) {
    read_file_bytes(path, dst, nbytes);
    return;
  }
  std::vector<char> v((size_t)nbytes);
  read_file_bytes(path, v.data(), nbytes);
  char* out = (char*)dst;
  for (int64_t c = 0; c < nc; ++c) {
    const char* src = v.data() + c * n_frames * sb;
    for (int64_t t = 0; t < n_frames; ++t) memcpy(out + (t * nc + c) * sb, src + t * sb, (size_t)sb);
  }
}

}  // namespace eegfx

using namespace eegfx;

extern "C" {

const char* eegfx_last_error(void) { return last_error().c_str(); }

int eegfx_read_header(const char* vhdr_path, eegfx_header_info* info, eegfx_channel_info* channels,
                      int32_t max_channels) {
  return guarded([&] {
    if (!vhdr_path || !info) fail(EEGFX_EINVAL, "null argument");
    Header h = read_header(vhdr_path);
    *info = h.info;
    if (channels)
      for (size_t i = 0; i < h.channels.size() && (int32_t)i < max_channels; ++i)
        channels[i] = h.channels[i];
  });
}

int eegfx_read_markers(const char* vmrk_path, eegfx_marker* markers, int64_t max_markers,
                       int64_t* n_markers) {
  return guarded([&] {
    if (!vmrk_path || !n_markers) fail(EEGFX_EINVAL, "null argument");
    std::vector<eegfx_marker> m = read_markers(vmrk_path);
    *n_markers = (int64_t)m.size();
    if (markers)
      for (size_t i = 0; i < m.size() && (int64_t)i < max_markers; ++i) markers[i] = m[i];
  });
}

int eegfx_recording_frames(const char* vhdr_path, const char* eeg_path, int64_t* n_frames) {
  return guarded([&] {
    if (!vhdr_path || !eeg_path || !n_frames) fail(EEGFX_EINVAL, "null argument");
    *n_frames = recording_frames(read_header(vhdr_path), eeg_path);
  });
}

int eegfx_plan_markers(const eegfx_marker* markers, int64_t n_markers, int64_t n_frames,
                       int32_t guessed, int64_t* balance, int64_t* pos_out, double* label_out,
                       int64_t* n_selected) {
  // Status is set explicitly (not via guarded) so that the accepted prefix survives an error,
  // like the epochs the reference has already appended when an exception aborts the loop.
  if (!balance || !n_selected || (n_markers > 0 && !markers)) {
    set_last_error("null argument");
    return EEGFX_EINVAL;
  }
  int64_t d = *balance, k = 0;
  for (int64_t i = 0; i < n_markers; ++i) {
    const eegfx_marker& m = markers[i];
    if (m.stimulus_index == INT32_MIN) {  // Integer.parseInt overflow (:212): uncaught NFE
      *balance = d;
      *n_selected = k;
      set_last_error(std::string("For input string: \"") + m.description + "\"");
      return EEGFX_EFORMAT;
    }
    const int64_t lo = m.position - EEGFX_PRESTIMULUS;
    if (lo < 0 || lo > n_frames) continue;  // Arrays.copyOfRange AIOOBE, caught at :262-264
    const bool target = (int64_t)m.stimulus_index + 1 == (int64_t)guessed;
    double label;
    if (target && d <= 0) {
      label = 1.0;
      ++d;
    } else if (!target && d >= 0) {
      label = 0.0;
      --d;
    } else {
      continue;
    }
    if (pos_out) pos_out[k] = m.position;
    if (label_out) label_out[k] = label;
    ++k;
  }
  *balance = d;
  *n_selected = k;
  set_last_error("");
  return EEGFX_OK;
}

}  // extern "C"
