"""yalantinglibs_amd — MI355X-native struct_pack batch codec.

The hot path (struct_pack serialize/deserialize of record batches) runs in
hand-written gfx950 HIP kernels behind the C ABI of include/spk_codec.h.
Python modules here are the host-side mirror of the reference interface
(type model, layout descriptors, API entry points) plus bench/test helpers.
"""
__all__ = ["schema", "layout", "synth", "struct_pack"]
