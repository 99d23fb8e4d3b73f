// Native JPEG decode for the map_rows image path: a GIL-free host thread pool
// that decodes a chunk of JPEG cells straight into one page-locked ragged
// buffer (the layout kernels/image.hip ragged_prep_kernel reads).
//
// The Python path (ops/host_ops.decode_image, PIL) holds the GIL for its
// header parsing and array wrapping: on the MI355X box it tops out near
// 3.8k img/s whatever the thread count (profiles/r5_img/decode_bench.log),
// below the GPU's rate for the reference's VGG scoring graph
// (reference src/main/python/tensorframes_snippets/read_image.py:35-75,
// 147-167). Here the whole decode runs in C++ threads.
//
// libjpeg(-turbo) is loaded at run time (dlopen, no headers in the image);
// the few struct fields used are declared here and checked at run time
// against the file's own SOF header, so an ABI mismatch disables the path
// instead of corrupting memory. Any image the native path cannot take
// (not a JPEG, CMYK, a libjpeg warning such as truncated data) is reported
// back and decoded by the Python fallback, which keeps PIL's semantics.
#pragma once

#include <ATen/ATen.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace tfa {

struct JpegHeader {
  int height = 0, width = 0, components = 0;
  bool progressive = false;
};

// Parse the SOF marker of a JPEG stream (no decode). False when `data` is not
// a JPEG this decoder takes (baseline / extended / progressive Huffman).
bool jpeg_parse_header(const uint8_t* data, size_t len, JpegHeader* h);

// True when libjpeg could be loaded and its ABI matched (probed once).
bool jpeg_native_available(std::string* why = nullptr);

// What the probe found: the library's own version (JPEG_LIB_VERSION, read
// from the version-mismatch error jpeg_CreateDecompress raises) and
// decompressor struct size (the size-mismatch error), the soname loaded, and
// whether that (version, size) pair is a known layout (else `why`).
struct JpegLibInfo {
  bool ok;
  int version;
  int64_t struct_size;
  std::string soname, why;
};
JpegLibInfo jpeg_native_info();
// tests: see the loaded library as another version (0 = the real one)
void jpeg_force_version(int version);

// Decode one JPEG into `dst` (height x width x out_c uint8, row-major).
// out_c: 3 (RGB; grayscale files are replicated) or 1 (grayscale files only).
// Returns false (with a reason) on any error or libjpeg warning.
bool jpeg_decode_into(const uint8_t* data, size_t len, int out_c, uint8_t* dst, size_t dst_bytes,
                      std::string* err);

// One chunk of cells decoded asynchronously on the decode pool into
//   buf = [int64 offsets[n] | int32 hw[n][2] | pixels ...]   (page-locked)
// Construction parses every header (cells whose header does not parse make
// `header_ok` false and start no work) and queues one task per image; wait()
// blocks until all tasks ran and returns the indices that failed to decode
// (their pixel ranges are left for the caller to fill). `pinned`: page-locked
// buffer from the runtime's pinned pool (else ordinary host memory).
class JpegBatch {
 public:
  JpegBatch(std::vector<std::pair<const uint8_t*, size_t>> cells, int out_c, int threads, bool pinned);
  ~JpegBatch();
  JpegBatch(const JpegBatch&) = delete;
  JpegBatch& operator=(const JpegBatch&) = delete;

  bool header_ok() const { return header_ok_; }
  int bad_header() const { return bad_header_; }
  std::vector<int64_t> wait();
  at::Tensor buffer() const { return buf_; }
  int64_t meta_bytes() const { return meta_bytes_; }
  int64_t offsets_bytes() const { return static_cast<int64_t>(cells_.size()) * 8; }
  std::vector<int64_t> shape(int64_t i) const;  // {h, w, c}
  int64_t pixel_offset(int64_t i) const { return offs_.at(i); }

 private:
  std::vector<std::pair<const uint8_t*, size_t>> cells_;
  std::vector<JpegHeader> hdr_;
  std::vector<int64_t> offs_;
  int out_c_;
  bool header_ok_ = true;
  int bad_header_ = -1;
  int64_t meta_bytes_ = 0;
  at::Tensor buf_;
  std::mutex mu_;
  std::condition_variable cv_;
  int pending_ = 0;
  std::vector<int64_t> failed_;
};

// Decode-pool size (threads actually started so far).
int decode_pool_threads();

}  // namespace tfa
