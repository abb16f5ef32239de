// b2h_frame.h -- internal: super-chunks attached to a contiguous frame (b2h_frame.cpp), as the
// super-chunk code (b2h_schunk.cpp) sees them.
//
// An attached handle (blosc2_schunk_open*, blosc2_schunk_from_buffer(copy = false)) keeps a frame
// link in schunk->frame: the reference's blosc2_frame_s (blosc/frame.h:50-75) restated for a
// read-only handle.  Its chunk index schunk->data holds what needs no read -- the 32-byte special
// chunks and, for an in-memory frame, pointers into the frame -- and NULL for a chunk still on the
// frame file.  Every reader of a chunk goes through chunk_ptrs / link_get_chunk, which read the
// missing ones through the frame's IO backend.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/blosc2.h"

namespace b2h {

// A growable byte buffer that is never zero-filled (a frame read fills it): malloc'd, or pinned
// (hipHostMalloc) when the bytes go on to the device -- the staged decode H2Ds a run of chunks
// read off a frame file straight from it.
struct ReadBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool pinned = false;
  ReadBuf() = default;
  explicit ReadBuf(bool pin) : pinned(pin) {}
  ReadBuf(const ReadBuf&) = delete;
  ReadBuf& operator=(const ReadBuf&) = delete;
  ~ReadBuf() { release(); }
  void release() {
    if (p && pinned) (void)hipHostFree(p);
    else free(p);
    p = nullptr;
    cap = 0;
  }
  bool ensure(size_t n) {
    if (n <= cap) return true;
    if (pinned) {
      release();
      if (hipHostMalloc(reinterpret_cast<void**>(&p), n, hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        return false;
      }
    } else {
      uint8_t* q = static_cast<uint8_t*>(realloc(p, n));
      if (!q) return false;
      p = q;
    }
    cap = n;
    return true;
  }
};

// `n` bytes at `pos` of an open stream of a buffer backend (is_allocation_necessary) into `dst`:
// one read, or a few concurrent reads of >= 16 MiB each for a large one.  With `mu` (a user
// backend, whose thread safety is unknown) the reads are one at a time under the lock.
int io_read_par(const blosc2_io_cb* io, void* fp, int64_t pos, int64_t n, uint8_t* dst, std::mutex* mu);

// True when `s` is attached to a frame (schunk->frame holds a link).
bool frame_attached(const blosc2_schunk* s);

// Host pointers of chunks [c0, c0 + n): the chunk index where it holds them, else read through
// the frame's backend -- one read per run of adjacent chunks, into `hold` (a buffer backend) or
// in place (a mapping backend).  The pointers are valid until `hold` is reused or freed.
int chunk_ptrs(blosc2_schunk* s, int64_t c0, int32_t n, std::vector<const uint8_t*>* ptrs, ReadBuf* hold);

// frame_get_chunk (blosc/frame.c:3378-3530): chunk i of an attached handle; a chunk read from a
// frame file is malloc'd (*needs_free true), anything else is handed out in place.
int link_get_chunk(blosc2_schunk* s, int64_t i, uint8_t** chunk, bool* needs_free);

// Frees the link (and the chunk index) of an attached handle; closes its backend stream and calls
// the backend's destroy on its params (blosc/schunk.c:698-705).
void link_free(blosc2_schunk* s);

}  // namespace b2h
