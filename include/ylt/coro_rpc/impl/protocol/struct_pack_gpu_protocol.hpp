// struct_pack_gpu_protocol.hpp — coro_rpc serialize protocol whose batch
// payloads are encoded / decoded by the MI355X struct_pack codec.
//
// coro_rpc picks its payload codec through a protocol type with three
// statics (reference include/ylt/coro_rpc/impl/protocol/struct_pack_protocol.hpp:20-37),
// called by the handler executor to decode the argument tuple
// (rpc_execute.hpp:83,90,98) and to encode the return value
// (rpc_execute.hpp:140-175) and by context::response_msg (context.hpp:114-136).
// This protocol keeps that interface and the wire bytes: a handler whose one
// argument, or whose return value, is a std::vector<R> of records the GPU
// model covers (struct_pack::gpu::is_gpu_batch_v) goes through the HIP
// kernels; every other argument tuple / return type, and batches below the
// size thresholds (where a PCIe round trip costs more than the CPU codec),
// use the reference's struct_pack_protocol unchanged. A GPU-encoding server
// therefore talks to CPU clients and the other way round.
//
// Selecting it: a rpc_protocol whose
//   using supported_serialize_protocols = std::variant<struct_pack_gpu_protocol>;
// (coro_rpc_protocol.hpp:81) -- or call internal::execute<rpc_protocol,
// struct_pack_gpu_protocol, func> directly, as tests/cpp/test_gpu_protocol.cpp does.
#pragma once
#include <cstddef>
#include <string>
#include <string_view>
#include <tuple>
#include <type_traits>

#include <ylt/coro_rpc/impl/protocol/struct_pack_protocol.hpp>
#include <ylt/struct_pack_gpu.hpp>

namespace coro_rpc::protocol {

struct struct_pack_gpu_protocol {
  // Batches smaller than these go to the CPU codec. Process-wide knobs
  // (0 = always the GPU path for batch types).
  static inline std::size_t min_gpu_bytes = 1u << 20;     // decode: payload bytes
  static inline std::size_t min_gpu_records = 1u << 14;   // encode: records

  template <typename T>
  static bool deserialize_to(T &t, std::string_view buffer) {
    if constexpr (std::tuple_size_v<T> == 1) {
      using A = std::remove_cvref_t<std::tuple_element_t<0, T>>;
      if constexpr (struct_pack::gpu::is_gpu_batch_v<A>) {
        static_assert(struct_pack::gpu::hash_matches_reference<A>());
        if (buffer.size() >= min_gpu_bytes)
          return !struct_pack::gpu::deserialize_to(std::get<0>(t), buffer);
      }
    }
    return struct_pack_protocol::deserialize_to(t, buffer);
  }

  template <typename T>
  static std::string serialize(const T &t) {
    if constexpr (struct_pack::gpu::is_gpu_batch_v<T>) {
      static_assert(struct_pack::gpu::hash_matches_reference<T>());
      if (t.size() >= min_gpu_records) return struct_pack::gpu::serialize<std::string>(t);
    }
    return struct_pack_protocol::serialize(t);
  }

  static std::string serialize() { return struct_pack_protocol::serialize(); }
};

}  // namespace coro_rpc::protocol
