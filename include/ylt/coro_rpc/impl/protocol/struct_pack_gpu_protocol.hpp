// struct_pack_gpu_protocol.hpp — coro_rpc serialize protocol whose payloads
// are encoded / decoded by the MI355X struct_pack codec (struct_pack::gpu).
//
// coro_rpc picks its payload codec through a protocol type with three
// statics (reference include/ylt/coro_rpc/impl/protocol/struct_pack_protocol.hpp:20-37),
// called by the handler executor to decode the argument tuple
// (rpc_execute.hpp:83,90,98) and to encode the return value
// (rpc_execute.hpp:140-175) and by context::response_msg (context.hpp:114-136).
// This protocol keeps that interface, its argument shapes and the wire bytes,
// and runs every payload through struct_pack::gpu at any size:
//   * one argument A: a message of A (a std::vector<R> of records is one
//     VECTOR message, any other type one message);
//   * several arguments: one message of std::tuple<Args...>, the type the
//     reference client packs them as (coro_rpc_client.hpp:1405-1410,
//     get_args_type, struct_pack/reflection.hpp:64-67);
//   * the return value: a message of its type; a void handler's reply is
//     serialize(std::monostate{}), its header alone.
// A type the GPU front end cannot describe fails to compile (static_assert in
// struct_pack::gpu); there is no CPU codec behind this protocol. A
// GPU-encoding server talks to CPU clients and the other way round: the bytes
// are the reference's.
//
// Selecting it: a rpc_protocol whose
//   using supported_serialize_protocols = std::variant<struct_pack_gpu_protocol>;
// (coro_rpc_protocol.hpp:81) -- or call internal::execute<rpc_protocol,
// struct_pack_gpu_protocol, func> directly, as tests/cpp/test_gpu_protocol.cpp does.
#pragma once
#include <string>
#include <string_view>
#include <tuple>
#include <type_traits>
#include <variant>

#include <ylt/struct_pack_gpu.hpp>

namespace coro_rpc::protocol {

struct struct_pack_gpu_protocol {
  // the argument tuple of a handler (rpc_execute.hpp:78-99): one argument is
  // its own message, several are one std::tuple message
  template <typename T>
  static bool deserialize_to(T &t, std::string_view buffer) {
    if constexpr (std::tuple_size_v<T> == 1) {
      using A = std::remove_cvref_t<std::tuple_element_t<0, T>>;
#if SPK_GPU_WITH_REFERENCE
      static_assert(struct_pack::gpu::hash_matches_reference<A>());
#endif
      return !struct_pack::gpu::deserialize_to(std::get<0>(t), buffer);
    } else {
#if SPK_GPU_WITH_REFERENCE
      static_assert(struct_pack::gpu::hash_matches_reference<T>());
#endif
      return !struct_pack::gpu::deserialize_to(t, buffer);
    }
  }

  template <typename T>
  static std::string serialize(const T &t) {
#if SPK_GPU_WITH_REFERENCE
    static_assert(struct_pack::gpu::hash_matches_reference<T>());
#endif
    return struct_pack::gpu::serialize<std::string>(t);
  }

  // the reply of a void handler (struct_pack_protocol.hpp:34-36)
  static std::string serialize() {
    return struct_pack::gpu::serialize<std::string>(std::monostate{});
  }
};

}  // namespace coro_rpc::protocol
