// rtw_kernel_mesh.hip — the F_MESHES path-kernel variants (cow, monument, the other triangle worlds) in a
// translation unit of their own, so that the Makefile can build them with the iterative-ILP machine scheduler
// (KFLAGS_MESH) while every other variant keeps max-ILP: the kernel source is rtw_kernel.hip's, unchanged;
// RTW_MESH_TU leaves out its host side and its non-template kernels, which rtw_kernel.o defines.
#define RTW_MESH_TU 1
#include "rtw_kernel.hip"

namespace rtw {
Variant pick_mesh(bool count, uint32_t need, bool half, bool codes16) {
  return count ? pick5<true, F_MESHES>(need, half, codes16) : pick5<false, F_MESHES>(need, half, codes16);
}
}  // namespace rtw
