"""ctypes bindings for the two in-tree native libraries.

* ``libbcio.so``          host BAM decode/encode + byte-exact formatter (``include/bcio.h``)
* ``libbasecount_hip.so`` gfx950 HIP kernels behind the C-ABI (``include/basecount_hip.h``)

Both are built by ``__graft_entry__.build()`` (``make -C basecount_amd/csrc``).  Loading is
lazy; a missing library raises ``ImportError`` with the build command — there is no CPU
fallback for the GPU path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_libs: dict = {}


def _load(name: str) -> C.CDLL:
    lib = _libs.get(name)
    if lib is not None:
        return lib
    path = os.path.join(_HERE, name)
    if name == "libbcio.so" and os.environ.get("BASECOUNT_HOST_LIB_DIR"):
        # host-only code may be swapped for its sanitizer build (scripts/asan.sh); the HIP
        # library never is
        path = os.path.join(os.environ["BASECOUNT_HOST_LIB_DIR"], name)
    if not os.path.exists(path):
        raise ImportError(
            f"{name} is not built; run `make -C {os.path.join(_HERE, 'csrc')}` "
            "or `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = C.CDLL(path)
    _libs[name] = lib
    return lib


# ---------------------------------------------------------------------------------- bcio
class BcioRecords(C.Structure):
    _fields_ = [
        ("n", C.c_int64),
        ("tid", C.c_void_p),
        ("pos", C.c_void_p),
        ("flag", C.c_void_p),
        ("mapq", C.c_void_p),
        ("l_seq", C.c_void_p),
        ("qstart", C.c_void_p),
        ("qend", C.c_void_p),
        ("rec_err", C.c_void_p),
        ("cig_off", C.c_void_p),
        ("cigar", C.c_void_p),
        ("seq_off", C.c_void_p),
        ("seq", C.c_void_p),
        ("qual", C.c_void_p),
        ("seq_bytes", C.c_uint64),
        ("ref_span", C.c_void_p),
        ("seq_event", C.c_void_p),
        ("seq_event_bytes", C.c_uint64),
    ]


class BcioSelection(C.Structure):
    _fields_ = [
        ("n_accepted", C.c_int64),
        ("keyerror_ordinal", C.c_int64),
        ("keyerror_rec", C.c_int64),
        ("ref_beg", C.c_void_p),
        ("pos", C.c_void_p),
        ("cig_beg", C.c_void_p),
        ("cig_n", C.c_void_p),
        ("seq_nib", C.c_void_p),
        ("qlen", C.c_void_p),
        ("ordinal", C.c_void_p),
        ("rec", C.c_void_p),
        ("span", C.c_void_p),
    ]


class BcioWriteSpec(C.Structure):
    _fields_ = [
        ("n_refs", C.c_int32),
        ("ref_names", C.POINTER(C.c_char_p)),
        ("ref_lens", C.c_void_p),
        ("n", C.c_int64),
        ("tid", C.c_void_p),
        ("pos", C.c_void_p),
        ("flag", C.c_void_p),
        ("mapq", C.c_void_p),
        ("cig_off", C.c_void_p),
        ("cigar", C.c_void_p),
        ("l_seq", C.c_void_p),
        ("seq_off", C.c_void_p),
        ("seq", C.c_void_p),
        ("qual_off", C.c_void_p),
        ("qual", C.c_void_p),
        ("level", C.c_int),
        ("nthreads", C.c_int),
    ]


def bcio() -> C.CDLL:
    lib = _libs.get("libbcio.so")
    if lib is not None:
        return lib
    lib = _load("libbcio.so")
    lib.bcio_last_error.restype = C.c_char_p
    lib.bcio_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
    lib.bcio_close.argtypes = [C.c_void_p]
    lib.bcio_close.restype = None
    lib.bcio_n_refs.argtypes = [C.c_void_p]
    lib.bcio_n_refs.restype = C.c_int32
    lib.bcio_ref_name.argtypes = [C.c_void_p, C.c_int32]
    lib.bcio_ref_name.restype = C.c_char_p
    lib.bcio_ref_len.argtypes = [C.c_void_p, C.c_int32]
    lib.bcio_ref_len.restype = C.c_int64
    lib.bcio_get_records.argtypes = [C.c_void_p, C.POINTER(BcioRecords)]
    lib.bcio_select.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(BcioSelection)]
    lib.bcio_stream_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
    lib.bcio_stream_next.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_void_p)]
    lib.bcio_stream_records.argtypes = [C.c_void_p]
    lib.bcio_stream_records.restype = C.c_int64
    lib.bcio_stream_n_refs.argtypes = [C.c_void_p]
    lib.bcio_stream_n_refs.restype = C.c_int32
    lib.bcio_stream_ref_name.argtypes = [C.c_void_p, C.c_int32]
    lib.bcio_stream_ref_name.restype = C.c_char_p
    lib.bcio_stream_ref_len.argtypes = [C.c_void_p, C.c_int32]
    lib.bcio_stream_ref_len.restype = C.c_int64
    lib.bcio_stream_close.argtypes = [C.c_void_p]
    lib.bcio_stream_close.restype = None
    lib.bcio_find_ref_start.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_uint64)]
    lib.bcio_find_record.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_uint64)]
    lib.bcio_stream_open_range.argtypes = [C.c_char_p, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
    lib.bcio_write_bam.argtypes = [C.c_char_p, C.POINTER(BcioWriteSpec)]
    lib.bcio_seq_to_event.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int]
    lib.bcio_fmt_new.argtypes = [C.POINTER(C.c_void_p)]
    lib.bcio_fmt_free.argtypes = [C.c_void_p]
    lib.bcio_fmt_free.restype = None
    lib.bcio_fmt_rows.argtypes = [
        C.c_void_p, C.c_char_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
        C.c_void_p, C.c_int, C.c_int, C.c_int,
    ]
    lib.bcio_fmt_take.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    lib.bcio_fmt_pyround_float.argtypes = [C.c_double, C.c_int, C.c_char_p, C.c_int]
    lib.bcio_fmt_pyround_int.argtypes = [C.c_int64, C.c_int, C.c_char_p, C.c_int]
    return lib


def bcio_check(rc: int) -> None:
    if rc != 0:
        msg = bcio().bcio_last_error().decode(errors="replace")
        if rc == -1:
            raise OSError(msg)
        raise ValueError(f"bcio error {rc}: {msg}")
