// BigFile feature store -> host / HBM, natively.
//
// The reference reads LINAS frame features through basic/bigfile.py: feature.bin is n_rows x
// ndims float32 row-major (LINAS-engine/basic/bigfile.py:6-18); BigFile.read opens the file,
// sorts the requested rows and seeks/`array.fromfile`s them one by one (:23-56), and the video
// data set calls read_one -- one open + seek + list conversion -- per FRAME
// (LINAS-engine/util/tag_data_provider.py:330-337).  Here feature.bin is mapped once; a batch of
// row ids is gathered by a small thread team with plain memcpy (the page cache is the source),
// and the device variant streams the gathered rows through a double-buffered pinned staging
// area with hipMemcpyAsync on the handle's stream, so the copy of chunk k overlaps the gather of
// chunk k+1.  The Python mirror (cmve/linas/bigfile.py) keeps BigFile's API and parses
// shape.txt / id.txt; this file only moves bytes.
#include "cmve_internal.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <thread>
#include <vector>

struct cmve_bigfile {
  int fd = -1;
  const char* base = nullptr;
  size_t bytes = 0;
  int64_t n_rows = 0;
  int32_t dim = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};  // staging halves, for the device gather
};

namespace cmve {

// rows[k] -> out[k, :], split over `threads` contiguous slices of the request
static void gather_rows(const cmve_bigfile* bf, const int64_t* rows, int64_t n, float* out, int threads) {
  const size_t rb = (size_t)bf->dim * sizeof(float);
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) memcpy(out + k * bf->dim, bf->base + (size_t)rows[k] * rb, rb);
  };
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 64 + 1));
  if (threads <= 1) {
    work(0, n);
    return;
  }
  std::vector<std::thread> team;
  team.reserve(threads);
  const int64_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = t * per, hi = std::min(n, lo + per);
    if (lo < hi) team.emplace_back(work, lo, hi);
  }
  for (auto& th : team) th.join();
}

static int check_rows(const cmve_bigfile* bf, const int64_t* rows, int64_t n, const char* fn) {
  for (int64_t k = 0; k < n; ++k)
    CMVE_REQUIRE(rows[k] >= 0 && rows[k] < bf->n_rows, "%s: row %lld out of range [0, %lld)", fn,
                 (long long)rows[k], (long long)bf->n_rows);
  return CMVE_OK;
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_bigfile_open(const char* feature_bin, int64_t n_rows, int32_t dim, cmve_bigfile_t* out) {
  CMVE_REQUIRE(feature_bin && out, "cmve_bigfile_open: NULL argument");
  CMVE_REQUIRE(n_rows >= 0 && dim > 0, "cmve_bigfile_open: bad shape %lld x %d", (long long)n_rows, dim);
  const int fd = open(feature_bin, O_RDONLY);
  CMVE_REQUIRE(fd >= 0, "cmve_bigfile_open: cannot open %s", feature_bin);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    CMVE_REQUIRE(false, "cmve_bigfile_open: cannot stat %s", feature_bin);
  }
  const size_t need = (size_t)n_rows * (size_t)dim * sizeof(float);
  if ((size_t)st.st_size < need) {
    close(fd);
    CMVE_REQUIRE(false, "cmve_bigfile_open: %s holds %lld bytes, shape.txt says %lld x %d float32",
                 feature_bin, (long long)st.st_size, (long long)n_rows, dim);
  }
  void* map = nullptr;
  if (need > 0) {
    map = mmap(nullptr, need, PROT_READ, MAP_SHARED, fd, 0);
    if (map == MAP_FAILED) {
      close(fd);
      CMVE_REQUIRE(false, "cmve_bigfile_open: mmap of %s failed", feature_bin);
    }
  }
  cmve_bigfile* bf = new cmve_bigfile;
  bf->fd = fd;
  bf->base = (const char*)map;
  bf->bytes = need;
  bf->n_rows = n_rows;
  bf->dim = dim;
  *out = bf;
  return CMVE_OK;
}

extern "C" int cmve_bigfile_close(cmve_bigfile_t bf) {
  if (!bf) return CMVE_OK;
  for (hipEvent_t e : bf->ev)
    if (e) (void)hipEventDestroy(e);
  if (bf->base) munmap((void*)bf->base, bf->bytes);
  if (bf->fd >= 0) close(bf->fd);
  delete bf;
  return CMVE_OK;
}

extern "C" int cmve_bigfile_gather(cmve_bigfile_t bf, const int64_t* rows, int64_t n, float* out, int32_t threads) {
  CMVE_REQUIRE(bf && (n == 0 || (rows && out)), "cmve_bigfile_gather: NULL argument");
  int st = check_rows(bf, rows, n, "cmve_bigfile_gather");
  if (st) return st;
  gather_rows(bf, rows, n, out, threads);
  return CMVE_OK;
}

extern "C" int cmve_bigfile_gather_device(cmve_handle_t h, cmve_bigfile_t bf, const int64_t* rows, int64_t n,
                                          float* dst, float* staging, int64_t staging_rows, int32_t threads) {
  CMVE_REQUIRE(h && bf && (n == 0 || (rows && dst && staging)), "cmve_bigfile_gather_device: NULL argument");
  CMVE_REQUIRE(staging_rows >= 2, "cmve_bigfile_gather_device: staging must hold >= 2 rows (two halves)");
  int st = check_rows(bf, rows, n, "cmve_bigfile_gather_device");
  if (st) return st;
  if (n == 0) return CMVE_OK;
  for (auto& e : bf->ev)
    if (!e) CMVE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const int64_t half = staging_rows / 2;
  const size_t rb = (size_t)bf->dim * sizeof(float);
  bool used[2] = {false, false};
  for (int64_t k0 = 0, c = 0; k0 < n; k0 += half, ++c) {
    const int s = (int)(c & 1);
    const int64_t m = std::min(half, n - k0);
    float* buf = staging + (size_t)s * half * bf->dim;
    if (used[s]) CMVE_HIP(hipEventSynchronize(bf->ev[s]));  // the copy out of this half is done
    gather_rows(bf, rows + k0, m, buf, threads);
    CMVE_HIP(hipMemcpyAsync(dst + (size_t)k0 * bf->dim, buf, (size_t)m * rb, hipMemcpyHostToDevice, h->stream));
    CMVE_HIP(hipEventRecord(bf->ev[s], h->stream));
    used[s] = true;
  }
  return CMVE_OK;
}
