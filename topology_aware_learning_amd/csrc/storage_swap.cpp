// Exchange the device memory behind two torch storages (host code, no kernels).
//
// A device-resident driver keeps every client's parameters and buffers as views of one pool
// tensor per segment (arena.ModelPool.bind).  Double-buffered rounds (round.RoundExecutor,
// double_buffer=True) write the round's output into a second pool of the same shape, then
// exchange the two storages' data pointers: every view bound to the first pool now reads the
// round's output, and the second pool holds the previous state, the next round's destination.
// One pointer exchange per segment instead of a copy back or one re-pointing per parameter.
//
// The storages are named by their c10::StorageImpl addresses (Python: UntypedStorage._cdata).
// The DataPtrs move whole (pointer, allocator context, deleter), so each block is freed by its
// own allocator when the storage that holds it at that time dies.
#include <c10/core/StorageImpl.h>

#include <cstdint>
#include <utility>

extern "C" int32_t tal_swap_storage(void* a, void* b) {
  auto* sa = static_cast<c10::StorageImpl*>(a);
  auto* sb = static_cast<c10::StorageImpl*>(b);
  if (sa == nullptr || sb == nullptr || sa == sb) return 1;
  if (sa->nbytes() != sb->nbytes() || sa->device() != sb->device()) return 2;
  c10::DataPtr pa = sa->set_data_ptr(c10::DataPtr(nullptr, sa->device()));
  c10::DataPtr pb = sb->set_data_ptr(std::move(pa));
  sa->set_data_ptr(std::move(pb));
  return 0;
}
