// Native on-disk feature ingest (include/vge_ingest.h): npz = zip of .npy members
// (numpy savez / savez_compressed: stored or raw-deflate members, zip64 records as numpy writes them),
// decoded by a pool of host threads straight into the caller's frame-store buffers.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <sched.h>
#include <vector>

#include "../../include/vge_ingest.h"

namespace {

// ------------------------------------------------------------------ file mapping
struct Mapped {
  const uint8_t* p = nullptr;
  size_t n = 0;
  bool ok = false;
  explicit Mapped(const char* path) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return;
    struct stat st;
    if (::fstat(fd, &st) == 0 && st.st_size > 0) {
      void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m != MAP_FAILED) {
        p = static_cast<const uint8_t*>(m);
        n = (size_t)st.st_size;
        ok = true;
      }
    }
    ::close(fd);
  }
  ~Mapped() {
    if (ok) ::munmap(const_cast<uint8_t*>(p), n);
  }
  Mapped(const Mapped&) = delete;
  Mapped& operator=(const Mapped&) = delete;
};

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

// ------------------------------------------------------------------ zip central directory
struct Member {
  std::string name;
  uint16_t method = 0;  // 0 stored, 8 deflate
  uint64_t csize = 0, usize = 0;
  const uint8_t* data = nullptr;  // compressed bytes
};

bool zip_members(const Mapped& f, std::vector<Member>& out) {
  if (f.n < 22) return false;
  // end of central directory: the last 0x06054b50 within the trailing 64 KiB + 22 bytes
  size_t eocd = (size_t)-1;
  const size_t lo = f.n > 65557 ? f.n - 65557 : 0;
  for (size_t i = f.n - 22 + 1; i-- > lo;)
    if (rd32(f.p + i) == 0x06054b50u) {
      eocd = i;
      break;
    }
  if (eocd == (size_t)-1) return false;
  uint64_t entries = rd16(f.p + eocd + 10), cd_size = rd32(f.p + eocd + 12), cd_off = rd32(f.p + eocd + 16);
  if (entries == 0xFFFF || cd_size == 0xFFFFFFFFu || cd_off == 0xFFFFFFFFu) {  // zip64 locator before it
    if (eocd < 20 || rd32(f.p + eocd - 20) != 0x07064b50u) return false;
    const uint64_t z64 = rd64(f.p + eocd - 20 + 8);
    if (z64 > f.n || f.n - z64 < 56 || rd32(f.p + z64) != 0x06064b50u) return false;
    entries = rd64(f.p + z64 + 32);
    cd_size = rd64(f.p + z64 + 40);
    cd_off = rd64(f.p + z64 + 48);
  }
  // bounds checks in subtraction form: zip64 fields are 64-bit and a crafted file must not wrap them
  if (cd_off > f.n || cd_size > f.n - cd_off) return false;
  size_t q = (size_t)cd_off;
  for (uint64_t e = 0; e < entries; ++e) {
    if (q > f.n || f.n - q < 46 || rd32(f.p + q) != 0x02014b50u) return false;
    Member m;
    m.method = rd16(f.p + q + 10);
    uint64_t cs = rd32(f.p + q + 20), us = rd32(f.p + q + 24);
    const uint16_t nl = rd16(f.p + q + 28), xl = rd16(f.p + q + 30), cl = rd16(f.p + q + 32);
    uint64_t loff = rd32(f.p + q + 42);
    if (f.n - q - 46 < (size_t)nl + xl + cl) return false;
    m.name.assign(reinterpret_cast<const char*>(f.p + q + 46), nl);
    // zip64 extra field (id 1): the 0xFFFFFFFF fields in the order usize, csize, local header offset
    const uint8_t* x = f.p + q + 46 + nl;
    for (size_t k = 0; k + 4 <= xl;) {
      const uint16_t id = rd16(x + k), sz = rd16(x + k + 2);
      if (k + 4 + sz > xl) break;
      if (id == 1) {
        size_t o = k + 4;
        if (us == 0xFFFFFFFFu && o + 8 <= k + 4 + sz) { us = rd64(x + o); o += 8; }
        if (cs == 0xFFFFFFFFu && o + 8 <= k + 4 + sz) { cs = rd64(x + o); o += 8; }
        if (loff == 0xFFFFFFFFu && o + 8 <= k + 4 + sz) { loff = rd64(x + o); o += 8; }
      }
      k += 4 + sz;
    }
    if (loff > f.n || f.n - loff < 30 || rd32(f.p + loff) != 0x04034b50u) return false;
    const uint64_t hdr_len = 30 + (uint64_t)rd16(f.p + loff + 26) + rd16(f.p + loff + 28);
    if (f.n - loff < hdr_len) return false;
    const size_t data = (size_t)(loff + hdr_len);
    if (cs > f.n - data) return false;
    m.csize = cs;
    m.usize = us;
    m.data = f.p + data;
    out.push_back(std::move(m));
    q += 46 + nl + xl + cl;
  }
  return true;
}

// ------------------------------------------------------------------ npy header
struct NpyHeader {
  size_t header_bytes = 0;  // magic + lengths + dict
  int itemsize = 0;         // 4 (<f4) or 8 (<f8)
  std::vector<int64_t> shape;
  // element count; -1 when a dimension is negative or the product overflows int64 (a malformed header)
  int64_t count() const {
    int64_t c = 1;
    for (int64_t s : shape) {
      if (s < 0 || (s > 0 && c > INT64_MAX / s)) return -1;
      c *= s;
    }
    return c;
  }
};

// Parse from the first `n` bytes; returns false if malformed or if more bytes are needed (need > n).
bool parse_npy(const uint8_t* p, size_t n, NpyHeader& h, size_t& need) {
  need = 12;
  if (n < 10 || memcmp(p, "\x93NUMPY", 6) != 0) return false;
  const int major = p[6];
  size_t hl, start;
  if (major == 1) {
    hl = rd16(p + 8);
    start = 10;
  } else if (major == 2 || major == 3) {
    if (n < 12) return false;
    hl = rd32(p + 8);
    start = 12;
  } else {
    return false;
  }
  need = start + hl;
  if (n < need) return false;
  const std::string d(reinterpret_cast<const char*>(p + start), hl);
  const size_t dp = d.find("'descr'");
  if (dp == std::string::npos) return false;
  const size_t q1 = d.find('\'', d.find(':', dp));
  const size_t q2 = d.find('\'', q1 + 1);
  if (q1 == std::string::npos || q2 == std::string::npos) return false;
  const std::string descr = d.substr(q1 + 1, q2 - q1 - 1);
  if (descr == "<f4" || descr == "|f4" || descr == "=f4") h.itemsize = 4;
  else if (descr == "<f8" || descr == "|f8" || descr == "=f8") h.itemsize = 8;
  else return false;
  const size_t fp = d.find("'fortran_order'");
  if (fp == std::string::npos) return false;
  size_t fv = d.find(':', fp);
  if (fv == std::string::npos) return false;
  while (++fv < d.size() && d[fv] == ' ') {
  }
  if (d.compare(fv, 5, "False") != 0) return false;  // C order only
  const size_t sp = d.find("'shape'");
  const size_t l = d.find('(', sp), r = d.find(')', l);
  if (sp == std::string::npos || l == std::string::npos || r == std::string::npos) return false;
  h.shape.clear();
  const std::string s = d.substr(l + 1, r - l - 1);
  size_t k = 0;
  while (k < s.size()) {
    while (k < s.size() && (s[k] == ' ' || s[k] == ',')) ++k;
    if (k >= s.size()) break;
    char* end = nullptr;
    const long long v = strtoll(s.c_str() + k, &end, 10);
    if (end == s.c_str() + k || v < 0) return false;
    h.shape.push_back(v);
    k = (size_t)(end - s.c_str());
  }
  h.header_bytes = need;
  return true;
}

// ------------------------------------------------------------------ member readers
// Inflates (or copies) member m: first its npy header, then (if dst) its data into dst as float32
// (expected element count `want`, or any count if want < 0).
class MemberReader {
 public:
  explicit MemberReader(const Member& m) : m_(m) {}
  ~MemberReader() {
    if (inited_) inflateEnd(&zs_);
  }
  bool header(NpyHeader& h) {
    uint8_t* buf = head_;
    size_t got = 0, need = 12;
    while (true) {
      if (need > sizeof(head_)) return false;
      if (!pull(buf + got, need - got)) return false;
      got = need;
      if (parse_npy(buf, got, h, need)) break;
      if (need <= got) return false;  // malformed, not short
    }
    h_ = h;
    return true;
  }
  bool data(float* dst, int64_t count) {
    if (count != h_.count()) return false;
    const size_t bytes = (size_t)count * h_.itemsize;
    if (h_.itemsize == 4) return pull(reinterpret_cast<uint8_t*>(dst), bytes);
    std::vector<double> tmp((size_t)count);
    if (!pull(reinterpret_cast<uint8_t*>(tmp.data()), bytes)) return false;
    for (int64_t i = 0; i < count; ++i) dst[i] = (float)tmp[(size_t)i];
    return true;
  }

 private:
  bool pull(uint8_t* out, size_t n) {  // next n bytes of the member's uncompressed stream
    if (n == 0) return true;
    if (m_.method == 0) {
      if (pos_ + n > m_.csize) return false;
      memcpy(out, m_.data + pos_, n);
      pos_ += n;
      return true;
    }
    if (m_.method != 8) return false;
    if (!inited_) {
      memset(&zs_, 0, sizeof(zs_));
      if (inflateInit2(&zs_, -15) != Z_OK) return false;
      inited_ = true;
      zs_.next_in = const_cast<Bytef*>(m_.data);
      zs_.avail_in = (uInt)std::min<uint64_t>(m_.csize, 0x7fffffffu);
      fed_ = zs_.avail_in;
    }
    zs_.next_out = out;
    zs_.avail_out = (uInt)n;
    while (zs_.avail_out > 0) {
      if (zs_.avail_in == 0 && fed_ < m_.csize) {  // members over 2 GiB: feed the rest
        const uint64_t rest = std::min<uint64_t>(m_.csize - fed_, 0x7fffffffu);
        zs_.next_in = const_cast<Bytef*>(m_.data + fed_);
        zs_.avail_in = (uInt)rest;
        fed_ += rest;
      }
      const int rc = inflate(&zs_, Z_NO_FLUSH);
      if (rc == Z_STREAM_END) return zs_.avail_out == 0;
      if (rc != Z_OK) return false;
    }
    return true;
  }
  const Member& m_;
  z_stream zs_;
  bool inited_ = false;
  uint64_t pos_ = 0, fed_ = 0;
  uint8_t head_[4096];
  NpyHeader h_;
};

const Member* find_member(const std::vector<Member>& ms, const char* key) {
  const std::string want = std::string(key) + ".npy";
  for (const Member& m : ms)
    if (m.name == want) return &m;
  return nullptr;
}

bool shape_is(const NpyHeader& h, std::initializer_list<int64_t> tail, int64_t* T) {
  if (h.shape.size() != tail.size() + 1) return false;
  size_t k = 1;
  for (int64_t d : tail)
    if (h.shape[k++] != d) return false;
  *T = h.shape[0];
  return true;
}

// keypoints.npy: a plain (uncompressed) .npy file, [T',120] (any shape with 120 per row accepted)
int kp_probe(const char* path, int32_t* rows, NpyHeader* hdr, Mapped** keep) {
  *rows = -1;
  if (!path) return VGE_INGEST_OK;
  if (::access(path, F_OK) != 0) return VGE_INGEST_OK;  // absent: the caller decides
  Mapped* f = new Mapped(path);
  if (!f->ok) {
    delete f;
    return VGE_INGEST_ERR_KP;
  }
  NpyHeader h;
  size_t need = 0;
  if (!parse_npy(f->p, f->n, h, need) || h.shape.empty() || h.count() < 0 || h.count() % 120 != 0 ||
      h.header_bytes > f->n || (uint64_t)h.count() > (f->n - h.header_bytes) / (uint64_t)h.itemsize) {
    delete f;
    return VGE_INGEST_ERR_KP;
  }
  *rows = (int32_t)(h.count() / 120);
  if (hdr) *hdr = h;
  if (keep) *keep = f;
  else delete f;
  return VGE_INGEST_OK;
}

int probe_one(const char* npz, const char* kpp, vge_clip_info* info) {
  info->n_frames = 0;
  info->vit_dim = 0;
  info->kp_frames = -1;
  Mapped f(npz);
  std::vector<Member> ms;
  if (!f.ok || !zip_members(f, ms)) return VGE_INGEST_ERR_IO;
  const Member* mp = find_member(ms, "pose");
  const Member* mv = find_member(ms, "vit");
  if (!mp || !mv) return VGE_INGEST_ERR_IO;
  NpyHeader hp, hv;
  MemberReader rp(*mp), rv(*mv);
  int64_t T = 0;
  if (!rp.header(hp) || !rv.header(hv)) return VGE_INGEST_ERR_IO;
  if (!shape_is(hp, {23, 3, 3}, &T) || hv.shape.size() != 2 || hv.shape[0] != T) return VGE_INGEST_ERR_SHAPE;
  if (T < 0 || T > INT32_MAX || hv.shape[1] <= 0 || hv.shape[1] > (1 << 20)) return VGE_INGEST_ERR_SHAPE;  // crafted sizes
  info->n_frames = (int32_t)T;
  info->vit_dim = (int32_t)hv.shape[1];
  int32_t rows = -1;
  const int kr = kp_probe(kpp, &rows, nullptr, nullptr);
  info->kp_frames = rows;
  return kr;
}

int decode_one(const char* npz, const char* kpp, const int32_t* vid, int vit_dim, float* pose, float* gori,
               float* betas, float* vit, float* kp) {
  Mapped f(npz);
  std::vector<Member> ms;
  if (!f.ok || !zip_members(f, ms)) return VGE_INGEST_ERR_IO;
  const int64_t off = vid[0], T = vid[1];
  struct Want {
    const char* key;
    std::initializer_list<int64_t> tail;
    float* dst;
    int64_t width;
  };
  const Want wants[4] = {{"pose", {23, 3, 3}, pose, 207},
                         {"global_orient", {1, 3, 3}, gori, 9},
                         {"betas", {10}, betas, 10},
                         {"vit", {(int64_t)vit_dim}, vit, (int64_t)vit_dim}};
  for (const Want& w : wants) {
    const Member* m = find_member(ms, w.key);
    if (!m) return VGE_INGEST_ERR_IO;
    MemberReader r(*m);
    NpyHeader h;
    int64_t t = 0;
    if (!r.header(h)) return VGE_INGEST_ERR_IO;
    if (!shape_is(h, w.tail, &t) || t != T) return VGE_INGEST_ERR_SHAPE;
    if (!r.data(w.dst + off * w.width, T * w.width)) return VGE_INGEST_ERR_IO;
  }
  const int64_t koff = vid[2], kT = vid[3];
  if (kT > 0) {
    Mapped* kf = nullptr;
    NpyHeader h;
    int32_t rows = -1;
    const int kr = kp_probe(kpp, &rows, &h, &kf);
    if (kr != VGE_INGEST_OK || rows != kT) {
      delete kf;
      return kr != VGE_INGEST_OK ? kr : VGE_INGEST_ERR_KP;
    }
    const uint8_t* src = kf->p + h.header_bytes;
    float* dst = kp + koff * 120;
    if (h.itemsize == 4) {
      memcpy(dst, src, (size_t)kT * 120 * 4);
    } else {
      for (int64_t i = 0; i < kT * 120; ++i) {
        double v;
        memcpy(&v, src + 8 * i, 8);
        dst[i] = (float)v;
      }
    }
    delete kf;
  }
  return VGE_INGEST_OK;
}

// CPU share of this process: the cgroup v2 quota (cpu.max "quota period") when one is set, else the
// affinity mask, else hardware_concurrency (which can count a whole many-socket machine).
int cpu_share() {
  cpu_set_t set;
  int n = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long long period = 0;
    if (fscanf(f, "%31s %lld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
      long long q = atoll(quota);
      if (q > 0) n = std::min<long long>(n, std::max<long long>(1, (q + period - 1) / period));
    }
    fclose(f);
  }
  return std::max(1, n);
}

// Decode threads per call: VGE_INGEST_THREADS, else OMP_NUM_THREADS when it asks for more than one thread
// (torchrun exports OMP_NUM_THREADS=1 for nproc_per_node > 1, which must not serialise the decoder), else
// this process's CPU share divided among the ranks of this node (LOCAL_WORLD_SIZE).  At most 64.
int default_threads() {
  if (const char* e = getenv("VGE_INGEST_THREADS"))
    if (atoi(e) > 0) return std::min(atoi(e), 64);
  if (const char* e = getenv("OMP_NUM_THREADS"))
    if (atoi(e) > 1) return std::min(atoi(e), 64);
  int n = cpu_share();
  if (const char* e = getenv("LOCAL_WORLD_SIZE"))
    if (atoi(e) > 1) n = std::max(1, n / atoi(e));
  return std::max(1, std::min(n, 64));
}

}  // namespace

extern "C" int vge_ingest_default_threads(void) { return default_threads(); }

namespace {

template <class Fn>
void parallel_for(int n, int n_threads, Fn fn) {
  int T = n_threads > 0 ? n_threads : default_threads();
  T = std::max(1, std::min(T, n));
  if (T == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  pool.reserve((size_t)T);
  for (int t = 0; t < T; ++t)
    pool.emplace_back([&]() {
      for (int i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (std::thread& th : pool) th.join();
}

}  // namespace

extern "C" {

int vge_ingest_probe(const char* const* npz_paths, const char* const* kp_paths, int n, int n_threads,
                     vge_clip_info* info) {
  if (n < 0 || (n > 0 && (!npz_paths || !info))) return VGE_INGEST_ERR_ARG;
  parallel_for(n, n_threads, [&](int i) {
    info[i].status = npz_paths[i] ? probe_one(npz_paths[i], kp_paths ? kp_paths[i] : nullptr, &info[i])
                                  : VGE_INGEST_ERR_ARG;
  });
  for (int i = 0; i < n; ++i)
    if (info[i].status != VGE_INGEST_OK) return info[i].status;
  return VGE_INGEST_OK;
}

int vge_ingest_decode(const char* const* npz_paths, const char* const* kp_paths, int n, int n_threads,
                      const int32_t* videos, int vit_dim, float* pose, float* gori, float* betas, float* vit,
                      float* kp, int32_t* status) {
  if (n < 0 || vit_dim < 1 || (n > 0 && (!npz_paths || !videos || !pose || !gori || !betas || !vit)))
    return VGE_INGEST_ERR_ARG;
  for (int i = 0; i < n; ++i)
    if (videos[4 * i + 3] > 0 && !kp) return VGE_INGEST_ERR_ARG;
  std::vector<int32_t> st((size_t)n, VGE_INGEST_OK);
  parallel_for(n, n_threads, [&](int i) {
    st[(size_t)i] = npz_paths[i] ? decode_one(npz_paths[i], kp_paths ? kp_paths[i] : nullptr, videos + 4 * i,
                                              vit_dim, pose, gori, betas, vit, kp)
                                 : VGE_INGEST_ERR_ARG;
  });
  int rc = VGE_INGEST_OK;
  for (int i = 0; i < n; ++i) {
    if (status) status[i] = st[(size_t)i];
    if (rc == VGE_INGEST_OK) rc = st[(size_t)i];
  }
  return rc;
}

}  // extern "C"
