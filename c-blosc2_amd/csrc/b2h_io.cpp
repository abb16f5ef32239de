// b2h_io.cpp -- the IO backend registry and the two built-in backends (host code only).
//
// The reference reads and writes frames through a table of callbacks (blosc2_io_cb,
// include/blosc2.h:1007-1041) looked up by id: the filesystem backend (blosc/blosc2-stdio.c:120-300)
// is id 0, the memory-mapped one (blosc2-stdio.c:330-560) id 1, and users register ids >= 160
// (blosc/blosc2.c:6784-6847).  Frame-attached super-chunks (b2h_frame.cpp) read their chunks
// through the entry their udio names, so a user backend sees every read.
//
// Filesystem reads and writes are positioned (pread / pwrite, looped over short transfers), so one
// open handle serves the fan-out's concurrent readers without a lock.  The mapped backend serves
// the read modes only ("r", "c"): reads hand out pointers into the mapping, which the chunk reader
// passes on without a copy.
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../../include/blosc2.h"

namespace {

bool trace_on() {
  static int on = -1;
  if (on < 0) on = getenv("BLOSC_TRACE") != nullptr;
  return on;
}
#define TRACE_ERROR(...)                                 \
  do {                                                   \
    if (trace_on()) {                                    \
      fprintf(stderr, "[error] - ");                     \
      fprintf(stderr, __VA_ARGS__);                      \
      fprintf(stderr, " (%s:%d)\n", __FILE__, __LINE__); \
    }                                                    \
  } while (0)

// size * nitems as a byte count, refusing negatives and overflow (blosc2-stdio.c checked_mul).
bool byte_count(int64_t size, int64_t nitems, int64_t* n) {
  if (size < 0 || nitems < 0) return false;
  if (size && nitems > INT64_MAX / size) return false;
  *n = size * nitems;
  return true;
}

// Positioned transfer of n bytes, looped over short counts and EINTR; returns the bytes moved.
int64_t pio(int fd, uint8_t* p, int64_t n, int64_t pos, bool write) {
  int64_t done = 0;
  while (done < n) {
    const size_t step = (size_t)std::min<int64_t>(n - done, int64_t(1) << 30);
    const ssize_t r = write ? pwrite(fd, p + done, step, (off_t)(pos + done)) : pread(fd, p + done, step, (off_t)(pos + done));
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (r == 0) break;
    done += r;
  }
  return done;
}

std::mutex g_io_mu;
blosc2_io_cb g_ios[256];
int g_nio = 0;

blosc2_io_cb stdio_cb() {
  blosc2_io_cb c{};
  c.id = BLOSC2_IO_FILESYSTEM;
  c.name = const_cast<char*>("filesystem");
  c.is_allocation_necessary = true;
  c.open = blosc2_stdio_open;
  c.close = blosc2_stdio_close;
  c.size = blosc2_stdio_size;
  c.write = blosc2_stdio_write;
  c.read = blosc2_stdio_read;
  c.truncate = blosc2_stdio_truncate;
  c.destroy = blosc2_stdio_destroy;
  return c;
}

blosc2_io_cb mmap_cb() {
  blosc2_io_cb c{};
  c.id = BLOSC2_IO_FILESYSTEM_MMAP;
  c.name = const_cast<char*>("filesystem_mmap");
  c.is_allocation_necessary = false;
  c.open = blosc2_stdio_mmap_open;
  c.close = blosc2_stdio_mmap_close;
  c.size = blosc2_stdio_mmap_size;
  c.write = blosc2_stdio_mmap_write;
  c.read = blosc2_stdio_mmap_read;
  c.truncate = blosc2_stdio_mmap_truncate;
  c.destroy = blosc2_stdio_mmap_destroy;
  return c;
}

// _blosc2_register_io_cb (blosc2.c:6784-6804): a known id with the same name is a no-op, with
// another name an error.  Caller holds g_io_mu.
int register_locked(const blosc2_io_cb* io) {
  for (int i = 0; i < g_nio; i++) {
    if (g_ios[i].id != io->id) continue;
    const char* a = g_ios[i].name ? g_ios[i].name : "";
    const char* b = io->name ? io->name : "";
    if (strcmp(a, b) != 0) {
      TRACE_ERROR("The IO (ID: %d) plugin is already registered with name: %s.  Choose another one !", io->id, a);
      return BLOSC2_ERROR_PLUGIN_IO;
    }
    return BLOSC2_ERROR_SUCCESS;
  }
  if (g_nio == 255) {
    TRACE_ERROR("Can not register more IO backends");
    return BLOSC2_ERROR_PLUGIN_IO;
  }
  g_ios[g_nio++] = *io;
  return BLOSC2_ERROR_SUCCESS;
}

}  // namespace

extern "C" {

int blosc2_register_io_cb(const blosc2_io_cb* io) {   // blosc2.c:6806-6819
  if (!io) return BLOSC2_ERROR_INVALID_PARAM;
  if (io->id < BLOSC2_IO_REGISTERED) {
    TRACE_ERROR("The compcode must be greater or equal than %d", BLOSC2_IO_REGISTERED);
    return BLOSC2_ERROR_PLUGIN_IO;
  }
  std::lock_guard<std::mutex> g(g_io_mu);
  return register_locked(io);
}

// blosc2.c:6821-6847: the built-in backends register themselves on first use.
blosc2_io_cb* blosc2_get_io_cb(uint8_t id) {
  std::lock_guard<std::mutex> g(g_io_mu);
  for (int i = 0; i < g_nio; i++)
    if (g_ios[i].id == id) return &g_ios[i];
  blosc2_io_cb builtin;
  if (id == BLOSC2_IO_FILESYSTEM) builtin = stdio_cb();
  else if (id == BLOSC2_IO_FILESYSTEM_MMAP) builtin = mmap_cb();
  else return nullptr;
  if (register_locked(&builtin) < 0) return nullptr;
  return &g_ios[g_nio - 1];
}

// ---------------------------------------------------------------- filesystem (stdio) ----
void* blosc2_stdio_open(const char* urlpath, const char* mode, void* params) {   // blosc2-stdio.c:136-156
  (void)params;
  if (!urlpath || !mode) {
    TRACE_ERROR("Invalid arguments for stdio open.");
    return nullptr;
  }
  FILE* f = fopen(urlpath, mode);
  if (!f) {
    TRACE_ERROR("Cannot open the file %s with mode %s.", urlpath, mode);
    return nullptr;
  }
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(malloc(sizeof(blosc2_stdio_file)));
  if (!h) {
    fclose(f);
    return nullptr;
  }
  h->file = f;
  return h;
}

int blosc2_stdio_close(void* stream) {
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(stream);
  if (!h || !h->file) return -1;
  const int rc = fclose(h->file);
  free(h);
  return rc;
}

int64_t blosc2_stdio_size(void* stream) {
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(stream);
  if (!h || !h->file) return -1;
  fflush(h->file);
  struct stat st;
  if (fstat(fileno(h->file), &st) != 0) return -1;
  return (int64_t)st.st_size;
}

int64_t blosc2_stdio_write(const void* ptr, int64_t size, int64_t nitems, int64_t position, void* stream) {
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(stream);
  int64_t n;
  if (!h || !h->file || !ptr || position < 0 || !byte_count(size, nitems, &n)) {
    TRACE_ERROR("Invalid arguments for stdio write.");
    return 0;
  }
  fflush(h->file);   // nothing buffered by stdio may land after (or over) the positioned write
  const int64_t done = pio(fileno(h->file), static_cast<uint8_t*>(const_cast<void*>(ptr)), n, position, true);
  const int64_t items = size > 0 ? done / size : 0;
  if (items != nitems) TRACE_ERROR("Short write at position %lld.", (long long)position);
  return items;
}

int64_t blosc2_stdio_read(void** ptr, int64_t size, int64_t nitems, int64_t position, void* stream) {
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(stream);
  int64_t n;
  if (!h || !h->file || !ptr || position < 0 || !byte_count(size, nitems, &n) || (n > 0 && !*ptr)) {
    TRACE_ERROR("Invalid arguments for stdio read.");
    return 0;
  }
  const int64_t done = pio(fileno(h->file), static_cast<uint8_t*>(*ptr), n, position, false);
  const int64_t items = size > 0 ? done / size : 0;
  if (items != nitems) TRACE_ERROR("Short read at position %lld.", (long long)position);
  return items;
}

int blosc2_stdio_truncate(void* stream, int64_t size) {
  blosc2_stdio_file* h = static_cast<blosc2_stdio_file*>(stream);
  if (!h || !h->file || size < 0) return -1;
  fflush(h->file);
  return ftruncate(fileno(h->file), (off_t)size) == 0 ? 0 : -1;
}

int blosc2_stdio_destroy(void* params) {
  (void)params;
  return 0;
}

// ------------------------------------------------------------------- memory-mapped ----
blosc2_stdio_mmap blosc2_get_blosc2_stdio_mmap_defaults(void) { return BLOSC2_STDIO_MMAP_DEFAULTS; }

// blosc2-stdio.c:330-470 for the read modes: the whole file mapped, PROT_READ and MAP_SHARED for
// "r", a private (copy-on-write) mapping for "c".  The params struct is the stream, as in the
// reference; opening the same params twice returns the live mapping.
void* blosc2_stdio_mmap_open(const char* urlpath, const char* mode, void* params) {
  (void)mode;   // the mapping mode comes from the params (blosc2-stdio.h:78)
  blosc2_stdio_mmap* m = static_cast<blosc2_stdio_mmap*>(params);
  if (!m || !urlpath) {
    TRACE_ERROR("The memory-mapped IO needs its blosc2_stdio_mmap params.");
    return nullptr;
  }
  if (m->addr) {
    if (!m->urlpath || strcmp(m->urlpath, urlpath) != 0) {
      TRACE_ERROR("The memory-mapped params already map %s.", m->urlpath ? m->urlpath : "?");
      return nullptr;
    }
    return m;
  }
  const char* md = m->mode ? m->mode : "";
  const bool copy_on_write = strcmp(md, "c") == 0;
  if (strcmp(md, "r") != 0 && !copy_on_write) {
    TRACE_ERROR("Mode %s: the memory-mapped backend opens existing frames for reading only (r, c).", md);
    return nullptr;
  }
  const int fd = open(urlpath, O_RDONLY);
  if (fd < 0) {
    TRACE_ERROR("Cannot open the file %s.", urlpath);
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size <= 0) {
    close(fd);
    TRACE_ERROR("Cannot map the (empty?) file %s.", urlpath);
    return nullptr;
  }
  const int prot = copy_on_write ? PROT_READ | PROT_WRITE : PROT_READ;
  const int flags = copy_on_write ? MAP_PRIVATE : MAP_SHARED;
  void* a = mmap(nullptr, (size_t)st.st_size, prot, flags, fd, 0);
  if (a == MAP_FAILED) {
    close(fd);
    TRACE_ERROR("Cannot map the file %s.", urlpath);
    return nullptr;
  }
  m->addr = static_cast<char*>(a);
  m->urlpath = strdup(urlpath);
  m->file_size = m->mapping_size = (size_t)st.st_size;
  m->is_memory_only = copy_on_write;
  m->file = nullptr;
  m->fd = fd;
  m->access_flags = prot;
  m->map_flags = flags;
  return m;
}

// The reference keeps the mapping open until destroy (blosc2-stdio.c:480-500): close is a no-op.
int blosc2_stdio_mmap_close(void* stream) {
  (void)stream;
  return 0;
}

int64_t blosc2_stdio_mmap_size(void* stream) {
  blosc2_stdio_mmap* m = static_cast<blosc2_stdio_mmap*>(stream);
  return m && m->addr ? (int64_t)m->file_size : -1;
}

int64_t blosc2_stdio_mmap_write(const void* ptr, int64_t size, int64_t nitems, int64_t position, void* stream) {
  (void)ptr; (void)size; (void)nitems; (void)position; (void)stream;
  TRACE_ERROR("The memory-mapped backend is read-only in the MI355X engine.");
  return 0;
}

// *ptr = the mapping at `position` (blosc2-stdio.c:520-545); the count is clipped at the file end.
int64_t blosc2_stdio_mmap_read(void** ptr, int64_t size, int64_t nitems, int64_t position, void* stream) {
  blosc2_stdio_mmap* m = static_cast<blosc2_stdio_mmap*>(stream);
  int64_t n;
  if (!m || !m->addr || !ptr || position < 0 || !byte_count(size, nitems, &n)) {
    TRACE_ERROR("Invalid arguments for mmap read.");
    return 0;
  }
  if (position > (int64_t)m->file_size) {
    *ptr = nullptr;
    return 0;
  }
  *ptr = m->addr + position;
  const int64_t avail = std::min<int64_t>(n, (int64_t)m->file_size - position);
  return size > 0 ? avail / size : 0;
}

int blosc2_stdio_mmap_truncate(void* stream, int64_t size) {
  blosc2_stdio_mmap* m = static_cast<blosc2_stdio_mmap*>(stream);
  return m && m->addr && size == (int64_t)m->file_size ? 0 : -1;
}

int blosc2_stdio_mmap_destroy(void* params) {
  blosc2_stdio_mmap* m = static_cast<blosc2_stdio_mmap*>(params);
  if (!m) return 0;
  int rc = 0;
  if (m->addr && munmap(m->addr, m->mapping_size) != 0) rc = -1;
  if (m->fd >= 0) close(m->fd);
  free(m->urlpath);
  m->addr = nullptr;
  m->urlpath = nullptr;
  m->fd = -1;
  m->file_size = m->mapping_size = 0;
  if (m->needs_free) free(m);
  return rc;
}

}  // extern "C"
