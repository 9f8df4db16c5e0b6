// shard.cpp — pre-decoded trial shards for the input path.
//
// Replaces, for this path, the reference's per-trial webdataset tars (src/prepare_data.py:210-235:
// `<eid>_<trial>.tar` holding `video.mp4` 120x128x128 gray + `ap.pyd` (100, N) spike counts) and
// its loader (src/loader/base.py:21-41: mp4 decode -> first channel -> (T, 1, H, W) -> `.float()`).
// The mp4 decode moves offline (once, at shard-writing time): a shard stores each trial's frames as
// raw uint8 (a quarter of the bytes the reference's float batch moves over PCIe, and what the K0
// kernel vs_video_preprocess reads directly) and its spike counts as f32, in fixed-size records so
// a batch is a set of positional reads straight into pinned host memory, split across threads.
//
// File layout (little-endian):
//   [0, 4096)       header: "VSSHARD1", u32 version, u32 n_records, u32 T, u32 C, u32 H, u32 W,
//                   u32 ap_rows, u32 ap_cols, u64 record_bytes, u64 data_offset, u64 video_bytes,
//                   u64 ap_bytes, u64 keys_offset
//   data_offset + i * record_bytes: record i = video u8 [T*C*H*W], zero pad to 4 KiB, ap f32
//                   [ap_rows*ap_cols], zero pad to 4 KiB
//   keys_offset:    n_records x 64-byte NUL-padded keys ("<eid>_<trial>", the webdataset __key__)
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "vspike.h"

namespace {

constexpr uint64_t kAlign = 4096;
constexpr char kMagic[8] = {'V', 'S', 'S', 'H', 'A', 'R', 'D', '1'};

struct Header {
  char magic[8];
  uint32_t version, n_records, T, C, H, W, ap_rows, ap_cols;
  uint64_t record_bytes, data_offset, video_bytes, ap_bytes, keys_offset;
};

struct Shard {
  int fd = -1;
  Header h{};
};

thread_local std::string g_err;

int fail(const char* msg) {
  g_err = msg;
  return VS_EINVAL;
}

uint64_t align_up(uint64_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

bool pread_all(int fd, void* dst, uint64_t n, uint64_t off) {
  char* p = (char*)dst;
  while (n > 0) {
    const ssize_t r = pread(fd, p, n, (off_t)off);
    if (r <= 0) return false;
    p += r;
    n -= (uint64_t)r;
    off += (uint64_t)r;
  }
  return true;
}

bool pwrite_all(int fd, const void* src, uint64_t n, uint64_t off) {
  const char* p = (const char*)src;
  while (n > 0) {
    const ssize_t r = pwrite(fd, p, n, (off_t)off);
    if (r <= 0) return false;
    p += r;
    n -= (uint64_t)r;
    off += (uint64_t)r;
  }
  return true;
}

}  // namespace

extern "C" const char* vs_shard_last_error(void) { return g_err.c_str(); }

extern "C" int vs_shard_write(const char* path, int64_t n, int64_t T, int64_t C, int64_t H, int64_t W,
                              int64_t ap_rows, int64_t ap_cols, const uint8_t* video, const float* ap,
                              const char* keys) {
  if (!path || n < 0 || T <= 0 || C <= 0 || H <= 0 || W <= 0 || ap_rows <= 0 || ap_cols <= 0)
    return fail("vs_shard_write: bad arguments");
  if (n > 0 && (!video || !ap || !keys)) return fail("vs_shard_write: null data");
  Header h{};
  memcpy(h.magic, kMagic, 8);
  h.version = 1;
  h.n_records = (uint32_t)n;
  h.T = (uint32_t)T; h.C = (uint32_t)C; h.H = (uint32_t)H; h.W = (uint32_t)W;
  h.ap_rows = (uint32_t)ap_rows; h.ap_cols = (uint32_t)ap_cols;
  h.video_bytes = (uint64_t)T * C * H * W;
  h.ap_bytes = (uint64_t)ap_rows * ap_cols * 4;
  h.record_bytes = align_up(h.video_bytes) + align_up(h.ap_bytes);
  h.data_offset = kAlign;
  h.keys_offset = h.data_offset + (uint64_t)n * h.record_bytes;
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return fail("vs_shard_write: cannot create file");
  std::vector<char> head(kAlign, 0);
  memcpy(head.data(), &h, sizeof(h));
  bool ok = pwrite_all(fd, head.data(), kAlign, 0);
  std::vector<char> rec(h.record_bytes, 0);
  for (int64_t i = 0; ok && i < n; ++i) {
    memcpy(rec.data(), video + i * h.video_bytes, h.video_bytes);
    memcpy(rec.data() + align_up(h.video_bytes), ap + i * (h.ap_bytes / 4), h.ap_bytes);
    ok = pwrite_all(fd, rec.data(), h.record_bytes, h.data_offset + (uint64_t)i * h.record_bytes);
  }
  if (ok && n > 0) ok = pwrite_all(fd, keys, (uint64_t)n * 64, h.keys_offset);
  if (close(fd) != 0) ok = false;
  return ok ? VS_OK : fail("vs_shard_write: write failed");
}

extern "C" void* vs_shard_open(const char* path, int64_t* info /* [8]: n, T, C, H, W, ap_rows, ap_cols, record_bytes */) {
  Shard* s = new Shard();
  s->fd = open(path, O_RDONLY);
  if (s->fd < 0) {
    fail("vs_shard_open: cannot open file");
    delete s;
    return nullptr;
  }
  struct stat st;
  if (!pread_all(s->fd, &s->h, sizeof(Header), 0) || memcmp(s->h.magic, kMagic, 8) != 0 || s->h.version != 1 ||
      fstat(s->fd, &st) != 0 || (uint64_t)st.st_size < s->h.keys_offset + (uint64_t)s->h.n_records * 64 ||
      s->h.record_bytes < s->h.video_bytes + s->h.ap_bytes) {
    fail("vs_shard_open: not a VSSHARD1 file (or truncated)");
    close(s->fd);
    delete s;
    return nullptr;
  }
  if (info) {
    const Header& h = s->h;
    const int64_t v[8] = {h.n_records, h.T, h.C, h.H, h.W, h.ap_rows, h.ap_cols, (int64_t)h.record_bytes};
    memcpy(info, v, sizeof(v));
  }
  return s;
}

extern "C" int vs_shard_key(void* handle, int64_t i, char* buf, int32_t n) {
  Shard* s = (Shard*)handle;
  if (!s || !buf || n < 65 || i < 0 || i >= (int64_t)s->h.n_records) return fail("vs_shard_key: bad arguments");
  if (!pread_all(s->fd, buf, 64, s->h.keys_offset + (uint64_t)i * 64)) return fail("vs_shard_key: read failed");
  buf[64] = 0;
  return VS_OK;
}

// Gather records idx[0..n) into video_dst [n, T*C*H*W] u8 and ap_dst [n, ap_rows*ap_cols] f32
// (pinned host buffers for an asynchronous H2D copy), `threads` readers in parallel.
extern "C" int vs_shard_read(void* handle, const int64_t* idx, int64_t n, uint8_t* video_dst, float* ap_dst,
                             int32_t threads) {
  Shard* s = (Shard*)handle;
  if (!s || (n > 0 && (!idx || !video_dst || !ap_dst)) || n < 0) return fail("vs_shard_read: bad arguments");
  for (int64_t k = 0; k < n; ++k)
    if (idx[k] < 0 || idx[k] >= (int64_t)s->h.n_records) return fail("vs_shard_read: record index out of range");
  const Header& h = s->h;
  const int nt = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  std::atomic<int64_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&]() {
    for (int64_t k = next++; k < n; k = next++) {
      const uint64_t base = h.data_offset + (uint64_t)idx[k] * h.record_bytes;
      if (!pread_all(s->fd, video_dst + k * h.video_bytes, h.video_bytes, base) ||
          !pread_all(s->fd, (char*)ap_dst + k * h.ap_bytes, h.ap_bytes, base + align_up(h.video_bytes)))
        ok = false;
    }
  };
  if (nt == 1 || n <= 1) {
    work();
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt && t < n; ++t) pool.emplace_back(work);
    for (auto& t : pool) t.join();
  }
  return ok ? VS_OK : fail("vs_shard_read: read failed");
}

extern "C" void vs_shard_close(void* handle) {
  Shard* s = (Shard*)handle;
  if (!s) return;
  if (s->fd >= 0) close(s->fd);
  delete s;
}
