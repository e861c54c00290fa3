"""Build the spk_layout descriptor (include/spk_codec.h) for a record type.

The descriptor carries the flattened COPY/SPAN ops plus the two message
formats the batch modes produce:
  fmt_vector — message type std::vector<T>  (SPK_MODE_VECTOR)
  fmt_one    — message type T               (SPK_MODE_MESSAGES)
each with its type code, type literal and resolved sp_config flags.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass
from typing import Optional

from . import _capi as C
from . import schema as S


@dataclass
class Layout:
    rtype: S.SpType
    dev: S.DeviceLayout
    c: C.spk_layout

    @property
    def ptr(self):
        return ct.byref(self.c)

    @property
    def stride(self):
        return self.dev.stride

    @property
    def n_spans(self):
        return len(self.dev.spans)

    @property
    def n_cont(self):
        """Members with a width-w count on the wire (SPAN: string / vector);
        an OPTION's 1-byte has_value and varints are in the plan's var_bytes."""
        from . import _capi as C
        if any(op[0] == C.SPK_OP_ARRAY for op in self.dev.ops):
            raise ValueError("count fields of an ARRAY layout depend on the data: "
                             "use parallel.count_fields(plan)")
        return sum(op[0] == C.SPK_OP_SPAN for op in self.dev.ops)


def make_layout(rtype: S.SpType, conf: int = S.DEFAULT, debug: bool = False,
                vector_config: Optional[int] = None) -> Layout:
    dev = S.flatten(rtype)
    L = C.spk_layout()
    L.abi = C.SPK_ABI_VERSION
    L.flags = C.SPK_LAYOUT_TRIVIAL if dev.trivial else 0
    L.rec_stride = dev.stride
    L.n_ops = len(dev.ops)
    for i, (k, o, s, a) in enumerate(dev.ops):
        L.ops[i].kind, L.ops[i].rec_off, L.ops[i].size, L.ops[i].aux = k, o, s, a
    vt = S.Vector(rtype, config=vector_config if vector_config is not None else S.DEFAULT)
    C.fill_msgfmt(L.fmt_vector, vt.code(), S.resolve_flags(vt, conf, debug), vt.root_literal())
    C.fill_msgfmt(L.fmt_one, rtype.code(), S.resolve_flags(rtype, conf, debug),
                  rtype.root_literal())
    return Layout(rtype, dev, L)


def case_layout(case: str, conf: int = S.DEFAULT, debug: bool = False) -> Layout:
    from . import synth
    return make_layout(synth.CASE_TYPES[case], conf, debug,
                       synth.VECTOR_CONFIG.get(case))
