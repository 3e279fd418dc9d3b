// mgp_buf.h — a u32 vector whose resize leaves new elements uninitialised (program
// buffers of hundreds of MB are written in full right after they are sized; zero-filling
// them first cost a serial pass over the memory).
#pragma once
#include <stdint.h>

#include <memory>
#include <vector>

template <typename T>
struct NoInitAlloc : std::allocator<T> {
  template <typename U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <typename U>
  NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
  template <typename U>
  void construct(U *p) noexcept {
    ::new (static_cast<void *>(p)) U;  // default-initialise: no zero fill
  }
  template <typename U, typename... Args>
  void construct(U *p, Args &&...args) {
    ::new (static_cast<void *>(p)) U(std::forward<Args>(args)...);
  }
};

typedef std::vector<uint32_t, NoInitAlloc<uint32_t>> U32Buf;
