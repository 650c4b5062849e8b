// orb_addrspace.h -- address-space-qualified pointers for the policy-templated algorithms.
//
// asp<AS, T> is T* in address space AS (3 = LDS, 1 = global), or a plain generic T* for
// AS = -1.  Kernels instantiate the octree/sort code with the spaces their buffers really live
// in, so the compiler emits ds_* / global_* instead of flat_* accesses (a flat access waits on
// both the LDS and the vector-memory counters); the host test harness uses -1.
#pragma once

namespace orbgpu {

template <int AS, class T>
struct asp_t {
    using type = __attribute__((address_space(AS))) T*;
};
template <class T>
struct asp_t<-1, T> {
    using type = T*;
};
template <int AS, class T>
using asp = typename asp_t<AS, T>::type;

constexpr int kGeneric = -1, kGlobalAS = 1, kLdsAS = 3;

// The 16-byte vector pointer in the same address space as P (whole-record ds_read_b128 /
// ds_write_b128 accesses of 16-byte records).
typedef unsigned int orb_u32x4 __attribute__((ext_vector_type(4)));
template <class P>
struct vec4_ptr;
template <class T>
struct vec4_ptr<T*> {
    using type = orb_u32x4*;
};
template <class T>
struct vec4_ptr<__attribute__((address_space(1))) T*> {
    using type = __attribute__((address_space(1))) orb_u32x4*;
};
template <class T>
struct vec4_ptr<__attribute__((address_space(3))) T*> {
    using type = __attribute__((address_space(3))) orb_u32x4*;
};
template <class T>
struct vec4_ptr<const T*> {
    using type = const orb_u32x4*;
};
template <class T>
struct vec4_ptr<const __attribute__((address_space(1))) T*> {
    using type = const __attribute__((address_space(1))) orb_u32x4*;
};
template <class T>
struct vec4_ptr<const __attribute__((address_space(3))) T*> {
    using type = const __attribute__((address_space(3))) orb_u32x4*;
};
template <class P>
__host__ __device__ inline typename vec4_ptr<P>::type as_vec4(P p) {
    return reinterpret_cast<typename vec4_ptr<P>::type>(p);
}

}  // namespace orbgpu
