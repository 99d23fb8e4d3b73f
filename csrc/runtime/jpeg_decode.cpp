// Native JPEG decode (see jpeg_decode.h). libjpeg(-turbo) entry points are
// resolved with dlopen; the decompressor struct is treated as opaque storage
// of the size the library reports, with the handful of leading fields this
// file reads or sets mirrored in DecompHead (their layout has not changed
// since libjpeg 6b; every value read is cross-checked).
#include "runtime/jpeg_decode.h"

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <csetjmp>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <thread>

#include "runtime/executor.h"

namespace tfa {

namespace {

// ---- the libjpeg ABI subset ------------------------------------------------
struct ErrorMgr {  // struct jpeg_error_mgr
  void (*error_exit)(void*);
  void (*emit_message)(void*, int);
  void (*output_message)(void*);
  void (*format_message)(void*, char*);
  void (*reset_error_mgr)(void*);
  int msg_code;
  union {
    int i[8];
    char s[80];
  } msg_parm;
  int trace_level;
  long num_warnings;
  const char* const* jpeg_message_table;
  int last_jpeg_message;
  const char* const* addon_message_table;
  int first_addon_message;
  int last_addon_message;
};

struct DecompHead {  // the leading fields of struct jpeg_decompress_struct
  ErrorMgr* err;
  void* mem;
  void* progress;
  void* client_data;
  int is_decompressor;
  int global_state;
  void* src;
  unsigned image_width, image_height;
  int num_components;
  int jpeg_color_space, out_color_space;
  unsigned scale_num, scale_denom;
  double output_gamma;
  int buffered_image, raw_data_out, dct_method, do_fancy_upsampling, do_block_smoothing;
  int quantize_colors, dither_mode, two_pass_quantize, desired_number_of_colors;
  int enable_1pass_quant, enable_external_quant, enable_2pass_quant;
  unsigned output_width, output_height;
  int out_color_components, output_components;
};
static_assert(offsetof(DecompHead, image_width) == 48, "libjpeg layout");
static_assert(offsetof(DecompHead, output_gamma) == 80, "libjpeg layout");
static_assert(offsetof(DecompHead, output_width) == 136, "libjpeg layout");
static_assert(offsetof(DecompHead, output_components) == 148, "libjpeg layout");

constexpr int JCS_GRAYSCALE = 1, JCS_RGB = 2;
constexpr size_t kStorage = 4096;  // >= sizeof(jpeg_decompress_struct) of any version

struct Lib {
  ErrorMgr* (*std_error)(ErrorMgr*) = nullptr;
  void (*create)(void*, int, size_t) = nullptr;
  void (*destroy)(void*) = nullptr;
  void (*mem_src)(void*, const unsigned char*, unsigned long) = nullptr;
  int (*read_header)(void*, int) = nullptr;
  int (*start)(void*) = nullptr;
  unsigned (*read_scanlines)(void*, unsigned char**, unsigned) = nullptr;
  int (*finish)(void*) = nullptr;
  int version = 0;
  size_t struct_size = 0;
  std::string soname;
  bool ok = false;
  std::string why;
};

// The (JPEG_LIB_VERSION, sizeof(jpeg_decompress_struct)) pairs of the LP64
// builds whose leading-field layout (DecompHead) has been verified: the
// library reported the pair itself and its decodes matched PIL bit for bit
// (tests/test_jpeg_native.py). Only libjpeg-turbo's libjpeg.so.8 (8 API) on
// this image so far; any other pair is refused and the Python decoder takes
// over (metric jpeg_native_unavailable), until it is verified and added here.
struct KnownLayout {
  int version;
  size_t struct_size;
};
constexpr KnownLayout kKnownLayouts[] = {{80, 656}};

bool known_layout(int version, size_t size) {
  for (const KnownLayout& k : kKnownLayouts)
    if (k.version == version && k.struct_size == size) return true;
  return false;
}

// tests: make the probe see another library version (0 = the real one)
std::atomic<int>& forced_version() {
  static std::atomic<int> v(0);
  return v;
}

struct Ctx {  // per-decode: error manager + jump buffer + the decompressor storage
  ErrorMgr err;
  jmp_buf jb;
  bool warned = false;
  char msg[200];
  alignas(16) unsigned char cinfo[kStorage];
};

Ctx* ctx_of(void* cinfo) {
  return reinterpret_cast<Ctx*>(reinterpret_cast<unsigned char*>(cinfo) - offsetof(Ctx, cinfo));
}

void on_error(void* cinfo) {
  Ctx* c = ctx_of(cinfo);
  if (c->err.format_message && c->err.jpeg_message_table) c->err.format_message(cinfo, c->msg);
  longjmp(c->jb, 1);
}

void on_message(void* cinfo, int level) {
  if (level < 0) ctx_of(cinfo)->warned = true;  // corrupt-data warning
}

void on_output(void*) {}

template <class F>
bool resolve(void* h, const char* name, F* fn, std::string* why) {
  *fn = reinterpret_cast<F>(dlsym(h, name));
  if (!*fn) *why = std::string("libjpeg symbol missing: ") + name;
  return *fn != nullptr;
}

Lib probe() {
  Lib L;
  void* h = nullptr;
  for (const char* name : {"libjpeg.so.8", "libjpeg.so.62", "libjpeg.so"}) {
    if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) {
      L.soname = name;
      break;
    }
  }
  if (!h) {
    L.why = "libjpeg not found";
    return L;
  }
  if (!resolve(h, "jpeg_std_error", &L.std_error, &L.why) || !resolve(h, "jpeg_CreateDecompress", &L.create, &L.why) ||
      !resolve(h, "jpeg_destroy_decompress", &L.destroy, &L.why) || !resolve(h, "jpeg_mem_src", &L.mem_src, &L.why) ||
      !resolve(h, "jpeg_read_header", &L.read_header, &L.why) ||
      !resolve(h, "jpeg_start_decompress", &L.start, &L.why) ||
      !resolve(h, "jpeg_read_scanlines", &L.read_scanlines, &L.why) ||
      !resolve(h, "jpeg_finish_decompress", &L.finish, &L.why))
    return L;
  // the library names its own version and struct size in the errors that
  // jpeg_CreateDecompress raises for a mismatching caller
  int version = 80;
  for (int attempt = 0; attempt < 2 && !L.struct_size; ++attempt) {
    auto c = std::make_unique<Ctx>();
    L.std_error(&c->err);
    c->err.error_exit = on_error;
    auto* head = reinterpret_cast<DecompHead*>(c->cinfo);
    head->err = &c->err;
    if (setjmp(c->jb) == 0) {
      L.create(c->cinfo, version, 0);  // size 0 never matches
      L.why = "libjpeg accepted a zero struct size";
      return L;
    }
    if (c->err.msg_parm.i[1] == 0 && c->err.msg_parm.i[0] > 0) {
      L.struct_size = static_cast<size_t>(c->err.msg_parm.i[0]);
    } else {
      version = c->err.msg_parm.i[0];  // version mismatch: the library's own version
    }
  }
  if (!L.struct_size || L.struct_size > kStorage || L.struct_size < sizeof(DecompHead)) {
    L.why = "libjpeg struct size probe failed";
    return L;
  }
  L.version = version;
  if (!known_layout(version, L.struct_size)) {
    L.why = "unknown libjpeg layout (version " + std::to_string(version) + ", decompressor struct " +
            std::to_string(L.struct_size) + " bytes)";
    return L;
  }
  L.ok = true;
  return L;
}

const Lib& probed() {
  static Lib L = probe();
  return L;
}

// the probed library, or (tests) the same library seen as another version,
// which the layout table then accepts or refuses
const Lib& lib() {
  const int fv = forced_version().load();
  if (fv == 0) return probed();
  thread_local Lib F;
  F = probed();
  F.version = fv;
  F.ok = F.struct_size && known_layout(fv, F.struct_size);
  if (!F.ok)
    F.why = "unknown libjpeg layout (version " + std::to_string(fv) + ", decompressor struct " +
            std::to_string(F.struct_size) + " bytes)";
  return F;
}

// ---- the decode pool --------------------------------------------------------
class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool();  // never destroyed: threads may outlive exit paths
    return *p;
  }
  void ensure(int n) {
    std::lock_guard<std::mutex> g(mu_);
    while (static_cast<int>(threads_.size()) < n) {
      threads_.emplace_back([this] { loop(); });
      threads_.back().detach();
    }
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() {
    std::lock_guard<std::mutex> g(mu_);
    return static_cast<int>(threads_.size());
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> threads_;
};

}  // namespace

bool jpeg_parse_header(const uint8_t* d, size_t n, JpegHeader* h) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return false;
  size_t i = 2;
  while (i + 3 < n) {
    if (d[i] != 0xFF) return false;
    uint8_t m = d[i + 1];
    if (m == 0xFF) {  // fill byte
      ++i;
      continue;
    }
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
      i += 2;
      continue;
    }
    size_t L = (static_cast<size_t>(d[i + 2]) << 8) | d[i + 3];
    if (L < 2 || i + 2 + L > n) return false;
    if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
      if (L < 8) return false;
      if (d[i + 4] != 8) return false;  // 8-bit samples only
      h->height = (d[i + 5] << 8) | d[i + 6];
      h->width = (d[i + 7] << 8) | d[i + 8];
      h->components = d[i + 9];
      h->progressive = m == 0xC2;
      return h->height > 0 && h->width > 0 && (h->components == 1 || h->components == 3);
    }
    if ((m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) || m == 0xD9 || m == 0xDA)
      return false;  // lossless / arithmetic / hierarchical, or data before a frame
    i += 2 + L;
  }
  return false;
}

bool jpeg_native_available(std::string* why) {
  const Lib& L = lib();
  if (why) *why = L.ok ? "libjpeg " + std::to_string(L.version) : L.why;
  return L.ok;
}

JpegLibInfo jpeg_native_info() {
  const Lib& L = lib();
  return {L.ok, L.version, static_cast<int64_t>(L.struct_size), L.soname, L.ok ? "" : L.why};
}

void jpeg_force_version(int version) { forced_version().store(version); }

bool jpeg_decode_into(const uint8_t* data, size_t len, int out_c, uint8_t* dst, size_t dst_bytes,
                      std::string* err) {
  const Lib& L = lib();
  if (!L.ok) {
    if (err) *err = L.why;
    return false;
  }
  JpegHeader hd;
  if (!jpeg_parse_header(data, len, &hd)) {
    if (err) *err = "not a supported JPEG";
    return false;
  }
  if (!(out_c == 3 || (out_c == 1 && hd.components == 1))) {
    if (err) *err = "unsupported channel conversion";
    return false;
  }
  const size_t row = static_cast<size_t>(hd.width) * out_c;
  if (dst_bytes < row * hd.height) {
    if (err) *err = "destination too small";
    return false;
  }
  auto c = std::make_unique<Ctx>();
  void* ci = c->cinfo;
  auto* head = reinterpret_cast<DecompHead*>(ci);
  L.std_error(&c->err);
  c->err.error_exit = on_error;
  c->err.emit_message = on_message;
  c->err.output_message = on_output;
  head->err = &c->err;
  volatile bool created = false;
  if (setjmp(c->jb)) {
    if (created) L.destroy(ci);
    if (err) *err = std::string("libjpeg: ") + c->msg;
    return false;
  }
  L.create(ci, L.version, L.struct_size);
  created = true;
  L.mem_src(ci, data, static_cast<unsigned long>(len));
  L.read_header(ci, 1);
  if (static_cast<int>(head->image_width) != hd.width || static_cast<int>(head->image_height) != hd.height ||
      head->num_components != hd.components) {
    L.destroy(ci);
    if (err) *err = "libjpeg header disagrees with the SOF marker";
    return false;
  }
  head->out_color_space = out_c == 3 ? JCS_RGB : JCS_GRAYSCALE;
  L.start(ci);
  if (static_cast<int>(head->output_width) != hd.width || static_cast<int>(head->output_height) != hd.height ||
      head->output_components != out_c) {
    L.destroy(ci);
    if (err) *err = "libjpeg output geometry disagrees";
    return false;
  }
  int y = 0;
  while (y < hd.height) {
    unsigned char* rows[8];
    int k = std::min(8, hd.height - y);
    for (int r = 0; r < k; ++r) rows[r] = dst + static_cast<size_t>(y + r) * row;
    unsigned got = L.read_scanlines(ci, rows, static_cast<unsigned>(k));
    if (got == 0) break;
    y += static_cast<int>(got);
  }
  if (y == hd.height) L.finish(ci);
  L.destroy(ci);
  if (y != hd.height || c->warned) {
    if (err) *err = c->warned ? "libjpeg warning (corrupt or truncated data)" : "short image";
    return false;
  }
  return true;
}

JpegBatch::JpegBatch(std::vector<std::pair<const uint8_t*, size_t>> cells, int out_c, int threads, bool pinned)
    : cells_(std::move(cells)), out_c_(out_c) {
  const int64_t n = static_cast<int64_t>(cells_.size());
  hdr_.resize(n);
  offs_.resize(n);
  int64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    JpegHeader& h = hdr_[i];
    if (!jpeg_parse_header(cells_[i].first, cells_[i].second, &h) ||
        !(out_c == 3 || (out_c == 1 && h.components == 1))) {
      header_ok_ = false;
      bad_header_ = static_cast<int>(i);
      return;
    }
    offs_[i] = total;
    total += static_cast<int64_t>(h.height) * h.width * out_c;
  }
  meta_bytes_ = n * 8 + n * 8;
  std::vector<int64_t> sz = {meta_bytes_ + std::max<int64_t>(total, 1)};
  buf_ = pinned ? empty_pinned(sz, at::kByte) : at::empty(sz, at::kByte);
  uint8_t* base = buf_.data_ptr<uint8_t>();
  std::memcpy(base, offs_.data(), n * 8);
  auto* hw = reinterpret_cast<int32_t*>(base + n * 8);
  for (int64_t i = 0; i < n; ++i) {
    hw[2 * i] = hdr_[i].height;
    hw[2 * i + 1] = hdr_[i].width;
  }
  if (n == 0) return;
  Pool::get().ensure(std::max(1, threads));
  pending_ = static_cast<int>(n);
  uint8_t* pix = base + meta_bytes_;
  for (int64_t i = 0; i < n; ++i) {
    Pool::get().submit([this, i, pix] {
      const JpegHeader& h = hdr_[i];
      size_t bytes = static_cast<size_t>(h.height) * h.width * out_c_;
      bool ok = jpeg_decode_into(cells_[i].first, cells_[i].second, out_c_, pix + offs_[i], bytes, nullptr);
      std::lock_guard<std::mutex> g(mu_);
      if (!ok) failed_.push_back(i);
      if (--pending_ == 0) cv_.notify_all();
    });
  }
}

JpegBatch::~JpegBatch() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [this] { return pending_ == 0; });  // tasks reference this object
}

std::vector<int64_t> JpegBatch::wait() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [this] { return pending_ == 0; });
  std::vector<int64_t> f = failed_;
  std::sort(f.begin(), f.end());
  return f;
}

std::vector<int64_t> JpegBatch::shape(int64_t i) const {
  const JpegHeader& h = hdr_.at(i);
  return {h.height, h.width, out_c_};
}

int decode_pool_threads() { return Pool::get().size(); }

}  // namespace tfa
