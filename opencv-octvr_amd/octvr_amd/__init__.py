"""Python binding of the MI355X octVR stitching library (include/octvr_hip.h) over ctypes.

Host-side mirror of the reference's octvr API for the stitching path:

* :class:`MapperTemplate`  <- ``vr::MapperTemplate`` (modules/octvr/include/octvr.hpp:47-91)
* :class:`Mapper`          <- ``vr::Mapper``         (modules/octvr/src/mapper.hpp:29-95)

Device buffers are torch tensors on ``cuda:N`` (PyTorch is plumbing here: allocation, streams,
torch.distributed); all arithmetic runs in the hand-written HIP kernels of ``liboctvr_hip.so``.
There is no CPU fallback: importing this module fails loudly when the library is missing.
"""
import ctypes as C
import json as _json
import os

import numpy as np
import torch  # must be imported first: the library then binds to torch's HIP runtime (one per process)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCTVR_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "liboctvr_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "liboctvr_hip.so not found at %s — build it with `make -C opencv-octvr_amd` or "
        "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)

_lib = C.CDLL(LIB_PATH)


# status codes of include/octvr_hip.h
E_INVALID, E_PARSE, E_HIP, E_UNSUPPORTED, E_IO = -1, -2, -3, -4, -5


class OctvrError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("octvr error %d: %s" % (code, msg))
        self.code = code


class InputView(C.Structure):
    _fields_ = [("roi_x", C.c_int), ("roi_y", C.c_int), ("roi_w", C.c_int), ("roi_h", C.c_int),
                ("map1", C.c_void_p), ("map2", C.c_void_p), ("mask", C.c_void_p), ("seam_mask", C.c_void_p),
                ("vignette", C.c_void_p), ("vignette_w", C.c_int), ("vignette_h", C.c_int)]


def _check(rc):
    if rc != 0:
        raise OctvrError(rc, _lib.octvr_last_error().decode())


_lib.octvr_last_error.restype = C.c_char_p
_VP = C.c_void_p
_lib.octvr_rig_create_json.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]
_lib.octvr_rig_load_dat.argtypes = [C.c_char_p, C.POINTER(_VP)]
_lib.octvr_rig_dump_dat.argtypes = [_VP, C.c_char_p]
_lib.octvr_rig_create_masks.argtypes = [_VP, C.c_int]
_lib.octvr_rig_create_from_arrays.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(_VP),
                                              C.POINTER(_VP), C.POINTER(_VP), C.POINTER(_VP), C.POINTER(_VP)]
_lib.octvr_rig_num_inputs.argtypes = [_VP, C.POINTER(C.c_int)]
_lib.octvr_rig_out_size.argtypes = [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int)]
_lib.octvr_rig_get_input.argtypes = [_VP, C.c_int, C.POINTER(InputView)]
_lib.octvr_rig_num_overlays.argtypes = [_VP, C.POINTER(C.c_int)]
_lib.octvr_rig_get_overlay.argtypes = [_VP, C.c_int, C.POINTER(InputView)]
_lib.octvr_rig_morph_controlpoints.argtypes = [_VP, C.c_char_p, C.POINTER(C.c_int)]
_lib.octvr_rig_get_triangles.argtypes = [_VP, C.c_int, _VP, _VP, C.c_int, C.POINTER(C.c_int)]
_lib.octvr_rig_destroy.argtypes = [_VP]
_lib.octvr_rig_destroy.restype = None
_lib.octvr_mapper_create.argtypes = [_VP, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int, C.c_int,
                                     C.c_int, C.c_int, C.POINTER(_VP)]
if hasattr(_lib, "octvr_mapper_create_ex"):
    _lib.octvr_mapper_create_ex.argtypes = [_VP, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                            C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]
REMAP_TEXTURE = 1  # octvr_hip.h OCTVR_REMAP_TEXTURE
_lib.octvr_mapper_stitch_batch.argtypes = [_VP, C.c_int, C.POINTER(_VP), C.POINTER(C.c_size_t), C.POINTER(_VP),
                                           C.c_size_t, _VP, _VP]
_lib.octvr_mapper_stitch_yuv420p.argtypes = [_VP, C.POINTER(_VP), C.POINTER(C.c_size_t), _VP, C.c_size_t,
                                             C.POINTER(C.c_double), C.c_int, _VP]
_lib.octvr_mapper_stitch_preview.argtypes = [_VP, C.POINTER(_VP), C.POINTER(C.c_size_t), _VP, C.c_size_t, _VP, C.c_int,
                                             C.c_int, C.c_size_t, C.POINTER(C.c_double), C.c_int, _VP]
_lib.octvr_mapper_gains.argtypes = [_VP, C.POINTER(C.c_double), C.c_int]
_lib.octvr_mapper_set_frames_in_flight.argtypes = [_VP, C.c_int]
_lib.octvr_mapper_traffic.argtypes = [_VP, C.POINTER(C.c_double)]
_lib.octvr_mapper_set_timing.argtypes = [_VP, C.c_int]
_lib.octvr_mapper_kernel_time.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_int)]
_lib.octvr_mapper_kernel_busy.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
_lib.octvr_mapper_kernel_intervals.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int,
                                               C.POINTER(C.c_int)]
_lib.octvr_rig_lut_recomputed.argtypes = [_VP, C.c_int, C.POINTER(C.c_uint64)]
_lib.octvr_debug_project_f64.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _VP, _VP, _VP]
_lib.octvr_interval_union.argtypes = [_VP, _VP, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
_lib.octvr_fastmapper_traffic.argtypes = [_VP, C.POINTER(C.c_double)]
_lib.octvr_mapper_info.argtypes = [_VP, C.c_char_p, C.c_size_t]
_lib.octvr_mapper_destroy.argtypes = [_VP]
_lib.octvr_mapper_destroy.restype = None
_lib.octvr_async_create.argtypes = [C.POINTER(_VP), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double),
                                    C.POINTER(_VP)]
if hasattr(_lib, "octvr_async_create_ex"):
    _lib.octvr_async_create_ex.argtypes = [C.POINTER(_VP), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                           C.POINTER(C.c_int), C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                           C.POINTER(C.c_double), C.c_int, C.POINTER(_VP)]
_lib.octvr_async_create_preview.argtypes = [C.POINTER(_VP), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                            C.POINTER(C.c_int), C.c_int, C.c_int, C.POINTER(C.c_int),
                                            C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int,
                                            C.POINTER(_VP)]


class PreviewDataHeader(C.Structure):
    """vr::PreviewDataHeader (octvr.hpp:97-101) = octvr_preview_header."""
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("step", C.c_int), ("fps", C.c_double)]


PREVIEW_SINK = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(PreviewDataHeader))
_lib.octvr_async_pop_preview.argtypes = [_VP, _VP, C.c_size_t, C.POINTER(PreviewDataHeader)]
_lib.octvr_async_set_preview_sink.argtypes = [_VP, PREVIEW_SINK, _VP]
_lib.octvr_async_info.argtypes = [_VP, C.c_char_p, C.c_size_t]
_lib.octvr_async_register_output.argtypes = [_VP, C.POINTER(_VP), C.POINTER(C.c_size_t)]
_lib.octvr_async_unregister_output.argtypes = [_VP, C.POINTER(_VP)]
_lib.octvr_async_push.argtypes = [_VP, C.POINTER(_VP), C.POINTER(C.c_size_t), C.POINTER(_VP), C.POINTER(C.c_size_t)]
_lib.octvr_async_pop.argtypes = [_VP]
_lib.octvr_async_pending.argtypes = [_VP, C.POINTER(C.c_int)]
_lib.octvr_async_destroy.argtypes = [_VP]
_lib.octvr_async_destroy.restype = None
_lib.octvr_fill_poly_u8.argtypes = [_VP, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int, C.c_uint8]
_lib.octvr_png_decode_rgb.argtypes = [C.c_char_p, C.c_size_t, _VP, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
_lib.octvr_fastmapper_create.argtypes = [_VP, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(_VP)]
_lib.octvr_fastmapper_stitch_nv12.argtypes = [_VP, C.POINTER(_VP), C.POINTER(C.c_size_t), _VP, C.c_size_t, _VP]
_lib.octvr_fastmapper_stitch_nv12_batch.argtypes = [_VP, C.c_int, C.POINTER(_VP), C.POINTER(C.c_size_t),
                                                    C.POINTER(_VP), C.c_size_t, _VP]
_lib.octvr_fastmapper_traffic_parts.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_double)]
_lib.octvr_mapper_traffic_parts.argtypes = [_VP, C.POINTER(C.c_double), C.POINTER(C.c_double)]
_lib.octvr_fastmapper_destroy.argtypes = [_VP]
_lib.octvr_fastmapper_destroy.restype = None
# self-test hooks (absent from older builds that OCTVR_HIP_LIB may select for an A/B)
if hasattr(_lib, "octvr_debug_json_number"):
    _lib.octvr_debug_json_number.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_double)]
if hasattr(_lib, "octvr_debug_tiled_lut_info"):
    _lib.octvr_debug_tiled_lut_info.argtypes = [_VP, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                                C.c_char_p, C.c_size_t]
if hasattr(_lib, "octvr_debug_fastmapper_audit"):
    _lib.octvr_debug_fastmapper_audit.argtypes = [_VP, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                                  C.c_int, C.c_char_p, C.c_size_t]
if hasattr(_lib, "octvr_debug_gain_plan"):
    _lib.octvr_debug_gain_plan.argtypes = [_VP, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int, _VP, _VP,
                                           C.c_size_t, C.POINTER(C.c_size_t)]
if hasattr(_lib, "octvr_debug_worker_failure"):
    _lib.octvr_debug_worker_failure.argtypes = [C.c_int, C.c_int]
_lib.octvr_remap_u8.argtypes = [_VP, C.c_int, C.c_int, C.c_size_t, C.c_int, _VP, _VP, C.c_int, C.c_int, C.c_size_t,
                                C.c_float, C.c_float, _VP, C.c_size_t, _VP]


def lib():
    return _lib


def abi_version():
    return _lib.octvr_abi_version()


def debug_project_f64(rig_json, out_w, out_h, input, device=0, where=0):
    """(x, y, fragile) — the FP64 projection of every output pixel for one input of a JSON rig, on the
    GPU (where=0; fragile = the LUT guard's verdict) or on the host with glibc (where=1; fragile None)
    (octvr_debug_project_f64)."""
    import numpy as _np
    x = _np.empty((out_h, out_w), _np.float64)
    y = _np.empty((out_h, out_w), _np.float64)
    f = _np.zeros((out_h, out_w), _np.uint8)
    _check(_lib.octvr_debug_project_f64(rig_json.encode() if isinstance(rig_json, str) else rig_json, out_w, out_h,
                                        int(input), int(device), int(where), x.ctypes.data_as(_VP),
                                        y.ctypes.data_as(_VP), f.ctypes.data_as(_VP)))
    return x, y, (f if where == 0 else None)


def debug_tiled_lut_info(mt, in_sizes, remap="remap"):
    """The blend = 0 composite's tiled LUT built on the host (octvr_debug_tiled_lut_info; no GPU), with its
    staged-group coverage check: a dict of items, wide tiles, staged / box pixels, bytes, histograms."""
    n = len(in_sizes)
    w = (C.c_int * n)(*[s[0] for s in in_sizes])
    h = (C.c_int * n)(*[s[1] for s in in_sizes])
    buf = C.create_string_buffer(4096)
    _check(_lib.octvr_debug_tiled_lut_info(mt._h, n, w, h, REMAP_TEXTURE if remap == "texture" else 0, buf, len(buf)))
    import json as _json
    return _json.loads(buf.value.decode())


def debug_worker_failure(n_threads, failing):
    """Run the host build's worker-thread helper with thread `failing` raising (octvr_debug_worker_failure;
    no GPU): raises OctvrError with the worker's message, as a failing tiler / seam / audit worker does."""
    _check(_lib.octvr_debug_worker_failure(int(n_threads), int(failing)))


def debug_gain_plan(mt, in_sizes, remap="remap"):
    """(entries, partners): the gain feed's samples as the mapper lays them out (octvr_debug_gain_plan; no
    GPU) — entries an (n, 2) uint32 array of (xy, code), partners a uint16 array."""
    import numpy as _np
    n = len(in_sizes)
    w = (C.c_int * n)(*[s[0] for s in in_sizes])
    h = (C.c_int * n)(*[s[1] for s in in_sizes])
    fl = REMAP_TEXTURE if remap == "texture" else 0
    cnt = C.c_size_t()
    _check(_lib.octvr_debug_gain_plan(mt._h, n, w, h, fl, None, None, 0, C.byref(cnt)))
    e = _np.zeros((cnt.value, 2), _np.uint32)
    p = _np.zeros(cnt.value, _np.uint16)
    _check(_lib.octvr_debug_gain_plan(mt._h, n, w, h, fl, e.ctypes.data, p.ctypes.data, cnt.value, C.byref(cnt)))
    return e, p


def debug_json_number(text, exact=True):
    """The first number of a JSON document as the rig-config reader parses it (octvr_debug_json_number):
    exact=True correctly rounded (OCTVR_JSON_EXACT), False with rapidjson's rules."""
    v = C.c_double()
    _check(_lib.octvr_debug_json_number(text.encode(), 1 if exact else 0, C.byref(v)))
    return v.value


def debug_fastmapper_audit(mt, in_sizes, wide=False, pitch_pad=0):
    """(ok, report): the host replay of every index the FastMapper kernels derive for this template and
    these input sizes, in the compact or (wide=True) 8-byte entry format (octvr_debug_fastmapper_audit;
    no GPU).  report: per plane ("y", "uv") the counts and the first violation."""
    n = len(in_sizes)
    w = (C.c_int * n)(*[s[0] for s in in_sizes])
    h = (C.c_int * n)(*[s[1] for s in in_sizes])
    buf = C.create_string_buffer(4096)
    rc = _lib.octvr_debug_fastmapper_audit(mt._h, n, w, h, int(bool(wide)), int(pitch_pad), buf, len(buf))
    import json as _json
    if not buf.value:  # the plan itself failed (bad arguments): no report
        _check(rc)
    return rc == 0, _json.loads(buf.value.decode())


def interval_union(starts, ends):
    """(summed lengths, length of the union) of the intervals [starts[k], ends[k]]
    (octvr_interval_union: the arithmetic of Mapper.kernel_busy)."""
    import numpy as _np
    a = _np.ascontiguousarray(starts, _np.float64)
    b = _np.ascontiguousarray(ends, _np.float64)
    sp, bu = C.c_double(), C.c_double()
    _check(_lib.octvr_interval_union(a.ctypes.data_as(_VP), b.ctypes.data_as(_VP), len(a), C.byref(sp), C.byref(bu)))
    return sp.value, bu.value


def _stream_ptr(stream):
    if isinstance(stream, C.c_void_p):
        return stream
    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


class MapperTemplate:
    """vr::MapperTemplate: JSON rig (LUT built on the GPU) or a VRv11 .dat file."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    @classmethod
    def from_json(cls, rig, out_w, out_h, use_roi=True, device=0):
        text = rig if isinstance(rig, str) else _json.dumps(rig)
        h = _VP()
        _check(_lib.octvr_rig_create_json(text.encode(), out_w, out_h, int(use_roi), device, C.byref(h)))
        return cls(h.value)

    @classmethod
    def load(cls, path):
        h = _VP()
        _check(_lib.octvr_rig_load_dat(os.fsencode(path), C.byref(h)))
        return cls(h.value)

    @classmethod
    def from_arrays(cls, out_w, out_h, rois, map1s, map2s, masks, seams=None):
        n = len(rois)
        map1s = [np.ascontiguousarray(a, np.float32) for a in map1s]
        map2s = [np.ascontiguousarray(a, np.float32) for a in map2s]
        masks = [np.ascontiguousarray(a, np.uint8) for a in masks]
        r = (C.c_int * (4 * n))(*[int(v) for roi in rois for v in roi])
        p1 = (_VP * n)(*[a.ctypes.data for a in map1s])
        p2 = (_VP * n)(*[a.ctypes.data for a in map2s])
        pm = (_VP * n)(*[a.ctypes.data for a in masks])
        ps = None
        if seams is not None:
            seams = [np.ascontiguousarray(a, np.uint8) for a in seams]
            ps = (_VP * n)(*[a.ctypes.data for a in seams])
        h = _VP()
        _check(_lib.octvr_rig_create_from_arrays(out_w, out_h, n, r, p1, p2, pm, ps, C.byref(h)))
        return cls(h.value)

    def dump(self, path):
        """MapperTemplate::dump: VRv11 file (creates the seam masks first if there are none)."""
        _check(_lib.octvr_rig_dump_dat(self._h, os.fsencode(path)))

    def lut_recomputed(self, i):
        """Output pixels of input i whose projection the GPU LUT build left to the host (glibc)."""
        n = C.c_uint64()
        _check(_lib.octvr_rig_lut_recomputed(self._h, i, C.byref(n)))
        return n.value

    def create_masks(self, device=0):
        """MapperTemplate::create_masks(): L2 distance seams (resizes on `device`)."""
        _check(_lib.octvr_rig_create_masks(self._h, device))

    def morph_controlpoints(self, control_points):
        """MapperTemplate::morph_controlpoints (template_morph.cpp:69-237): control_points is the rig
        JSON's "control_points" list of [n0, n1, x0, y0, x1, y1].  Returns the number kept."""
        text = control_points if isinstance(control_points, str) else _json.dumps(control_points)
        k = C.c_int()
        _check(_lib.octvr_rig_morph_controlpoints(self._h, text.encode(), C.byref(k)))
        return k.value

    def triangles(self, i):
        """inputs[i].src_triangles, dst_triangles of the last morph: two (n, 6) float32 arrays."""
        n = C.c_int()
        _check(_lib.octvr_rig_get_triangles(self._h, i, None, None, 0, C.byref(n)))
        src = np.zeros((n.value, 6), np.float32)
        dst = np.zeros((n.value, 6), np.float32)
        _check(_lib.octvr_rig_get_triangles(self._h, i, src.ctypes.data, dst.ctypes.data, n.value, C.byref(n)))
        return src, dst

    @property
    def out_size(self):
        w, h = C.c_int(), C.c_int()
        _check(_lib.octvr_rig_out_size(self._h, C.byref(w), C.byref(h)))
        return w.value, h.value

    def __len__(self):
        n = C.c_int()
        _check(_lib.octvr_rig_num_inputs(self._h, C.byref(n)))
        return n.value

    @property
    def num_overlays(self):
        n = C.c_int()
        _check(_lib.octvr_rig_num_overlays(self._h, C.byref(n)))
        return n.value

    def overlay(self, i):
        """Overlay input i (MapperTemplate::overlay_inputs): (roi, map1, map2, mask, None)."""
        return self.input(i, _overlay=True)

    def input(self, i, _overlay=False):
        """(roi, map1, map2, mask, seam_mask) as numpy copies."""
        v = InputView()
        _check((_lib.octvr_rig_get_overlay if _overlay else _lib.octvr_rig_get_input)(self._h, i, C.byref(v)))
        k = v.roi_w * v.roi_h
        shape = (v.roi_h, v.roi_w)

        def arr(ptr, ctype, dtype):
            if not ptr:
                return None
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), shape=(k,)).astype(dtype).reshape(shape)

        return ((v.roi_x, v.roi_y, v.roi_w, v.roi_h), arr(v.map1, C.c_float, np.float32),
                arr(v.map2, C.c_float, np.float32), arr(v.mask, C.c_uint8, np.uint8),
                arr(v.seam_mask, C.c_uint8, np.uint8))

    def vignette(self, i):
        """The input's vignette map (Vignette::getMap, vignette.cpp:39-54) or None."""
        v = InputView()
        _check(_lib.octvr_rig_get_input(self._h, i, C.byref(v)))
        if not v.vignette:
            return None
        k = v.vignette_w * v.vignette_h
        return np.ctypeslib.as_array(C.cast(v.vignette, C.POINTER(C.c_float)), shape=(k,)).copy().reshape(
            v.vignette_h, v.vignette_w)

    def close(self):
        if self._h and self._h.value:
            _lib.octvr_rig_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FrameRefs:
    """A frame set's device pointers and pitches marshalled once (Mapper.frame_refs), for callers that
    stitch the same buffers repeatedly (a capture ring): stitch() then skips the per-call ctypes work."""
    __slots__ = ("tensors", "ptrs", "pitches", "n")

    def __init__(self, tensors):
        self.tensors = list(tensors)  # kept alive while the references are in use
        self.n = len(self.tensors)
        self.ptrs = (_VP * self.n)(*[t.data_ptr() for t in self.tensors])
        self.pitches = (C.c_size_t * self.n)(*[t.stride(0) for t in self.tensors])


class BatchRefs:
    """Several frame sets' device pointers and their outputs marshalled once (Mapper.batch_refs)."""
    __slots__ = ("keep", "ptrs", "pitches", "outs", "out_pitch", "nf")

    def __init__(self, frame_sets, outputs):
        refs = [fs if isinstance(fs, FrameRefs) else FrameRefs(fs) for fs in frame_sets]
        self.nf = len(refs)
        assert len(outputs) == self.nf, "one output per frame set"
        self.keep = (refs, list(outputs))
        ptrs = [p for r in refs for p in r.ptrs]
        pitches = [p for r in refs for p in r.pitches]
        self.ptrs = (_VP * len(ptrs))(*ptrs)
        self.pitches = (C.c_size_t * len(pitches))(*pitches)
        self.outs = (_VP * self.nf)(*[o.data_ptr() for o in outputs])
        self.out_pitch = outputs[0].stride(0)
        assert all(o.stride(0) == self.out_pitch for o in outputs), "the outputs of a batch share one pitch"


class Mapper:
    """vr::Mapper on one device: stitch(inputs YUV420P, output YUV420P) with optional gain."""

    def __init__(self, mt, in_sizes, blend=0, enable_gain=True, device=0, scale_output=(0, 0), remap="remap"):
        """remap: "remap" (cv::remap's fixed point, the default) or "texture" (the reference's CUDA
        fastRemap texture sampling, OCTVR_REMAP_TEXTURE)."""
        n = len(in_sizes)
        w = (C.c_int * n)(*[s[0] for s in in_sizes])
        h = (C.c_int * n)(*[s[1] for s in in_sizes])
        scale_output = tuple(scale_output) if scale_output else (0, 0)  # None / () = unscaled
        if remap not in ("remap", "texture"):
            raise ValueError("remap must be 'remap' or 'texture'")
        hd = _VP()
        if remap == "texture":
            _check(_lib.octvr_mapper_create_ex(mt._h, device, n, w, h, blend, int(enable_gain), scale_output[0],
                                               scale_output[1], REMAP_TEXTURE, C.byref(hd)))
        else:
            _check(_lib.octvr_mapper_create(mt._h, device, n, w, h, blend, int(enable_gain), scale_output[0],
                                            scale_output[1], C.byref(hd)))
        self._h = hd
        self.n = n
        self.device = device
        # output frame size: scale_output, or the template's out_size (mapper.cpp:69)
        self.out_size = tuple(scale_output) if scale_output[0] else mt.out_size

    @staticmethod
    def frame_refs(inputs):
        """FrameRefs of a list of input tensors, accepted by stitch() in place of the list."""
        return FrameRefs(inputs)

    def stitch(self, inputs, output, gains=None, stream=None, preview=None):
        """inputs: list of uint8 cuda tensors (1.5H x W "Y over [U|V]") or their FrameRefs; output likewise.
        preview: an optional (h, w, 3) uint8 cuda tensor receiving Mapper::stitch's preview_output (the RGB
        result resized, mapper.cpp:308-312).  stream: a torch stream or a raw ctypes stream handle."""
        if isinstance(inputs, FrameRefs):
            n, ptrs, pitches = inputs.n, inputs.ptrs, inputs.pitches
        else:
            n = len(inputs)
            ptrs = (_VP * n)(*[t.data_ptr() for t in inputs])
            pitches = (C.c_size_t * n)(*[t.stride(0) for t in inputs])
        g = None
        ng = 0
        if gains is not None:
            g = (C.c_double * len(gains))(*gains)
            ng = len(gains)
        if preview is None:
            _check(_lib.octvr_mapper_stitch_yuv420p(self._h, ptrs, pitches, C.c_void_p(output.data_ptr()),
                                                    output.stride(0), g, ng, _stream_ptr(stream)))
        else:
            assert preview.dim() == 3 and preview.shape[2] == 3 and preview.stride(1) == 3 and preview.stride(2) == 1
            _check(_lib.octvr_mapper_stitch_preview(self._h, ptrs, pitches, C.c_void_p(output.data_ptr()),
                                                    output.stride(0), C.c_void_p(preview.data_ptr()),
                                                    preview.shape[1], preview.shape[0], preview.stride(0), g, ng,
                                                    _stream_ptr(stream)))

    @staticmethod
    def batch_refs(frame_sets, outputs):
        """BatchRefs of several frame sets (lists of input tensors or FrameRefs) and their outputs, accepted
        by stitch_batch() in place of the lists."""
        return BatchRefs(frame_sets, outputs)

    def stitch_batch(self, frame_sets, outputs=None, gains=None, stream=None):
        """len(frame_sets) (1, 2 or 4) frames in one call (octvr_mapper_stitch_batch): each frame's gains
        estimated (or gains: one list per frame), one composite launch for all; outputs: one tensor per
        frame (same pitch).  frame_sets may be a BatchRefs (outputs then None)."""
        b = frame_sets if isinstance(frame_sets, BatchRefs) else BatchRefs(frame_sets, outputs)
        g = None
        if gains is not None:
            flat = [float(v) for gl in gains for v in gl]
            g = (C.c_double * len(flat))(*flat)
        _check(_lib.octvr_mapper_stitch_batch(self._h, b.nf, b.ptrs, b.pitches, b.outs, b.out_pitch, g,
                                              _stream_ptr(stream)))

    def gains(self):
        g = (C.c_double * self.n)()
        _check(_lib.octvr_mapper_gains(self._h, g, self.n))
        return list(g)

    def set_frames_in_flight(self, k):
        """k slots of per-frame device state: stitches issued on different streams overlap
        (octvr_mapper_set_frames_in_flight).  No scaled output; multi-band / feather mappers get
        per-slot pyramids."""
        _check(_lib.octvr_mapper_set_frames_in_flight(self._h, int(k)))

    def traffic_bytes(self):
        b = C.c_double()
        _check(_lib.octvr_mapper_traffic(self._h, C.byref(b)))
        return b.value

    def traffic_parts(self):
        """(lut bytes read once per launch, bytes per frame) of the composite (octvr_mapper_traffic_parts)."""
        a, b = C.c_double(), C.c_double()
        _check(_lib.octvr_mapper_traffic_parts(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def info(self):
        buf = C.create_string_buffer(8192)
        _check(_lib.octvr_mapper_info(self._h, buf, 8192))
        return _json.loads(buf.value.decode())

    def set_timing(self, enable=True):
        _check(_lib.octvr_mapper_set_timing(self._h, int(enable)))

    def kernel_time(self):
        """(total device ms, launches) of the composite kernel since the last call (synchronizes)."""
        t, k = C.c_double(), C.c_int()
        _check(_lib.octvr_mapper_kernel_time(self._h, C.byref(t), C.byref(k)))
        return t.value, k.value

    def kernel_busy(self):
        """(summed start-to-end ms, union ms, launches) of the logged launches (synchronizes)."""
        sp, bu, k = C.c_double(), C.c_double(), C.c_int()
        _check(_lib.octvr_mapper_kernel_busy(self._h, C.byref(sp), C.byref(bu), C.byref(k)))
        return sp.value, bu.value, k.value

    def kernel_intervals(self, cap=4096):
        """[(start ms, end ms)] of the logged launches relative to the first one's start, in issue order
        (synchronizes; clears the log as kernel_busy does)."""
        st, en, k = (C.c_double * cap)(), (C.c_double * cap)(), C.c_int()
        _check(_lib.octvr_mapper_kernel_intervals(self._h, st, en, cap, C.byref(k)))
        return [(st[i], en[i]) for i in range(min(k.value, cap))]

    def close(self):
        if self._h and self._h.value:
            _lib.octvr_mapper_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FastMapper:
    """vr::FastMapper (modules/octvr/src/mapper_fast.cpp): feather-weighted NV12 stitch of a full-frame rig."""

    def __init__(self, mt, in_sizes, device=0):
        n = len(in_sizes)
        w = (C.c_int * n)(*[s[0] for s in in_sizes])
        h = (C.c_int * n)(*[s[1] for s in in_sizes])
        hd = _VP()
        _check(_lib.octvr_fastmapper_create(mt._h, device, n, w, h, C.byref(hd)))
        self._h = hd
        self.n = n
        self.out_size = mt.out_size

    def traffic_bytes(self):
        """Algorithmic bytes of one stitch_nv12 (octvr_fastmapper_traffic)."""
        b = C.c_double()
        _check(_lib.octvr_fastmapper_traffic(self._h, C.byref(b)))
        return b.value

    def stitch_nv12(self, inputs, output, stream=None):
        """inputs: uint8 cuda tensors (1.5H x W NV12) or their FrameRefs; output: 1.5H x W (chroma rows V,U)."""
        if isinstance(inputs, FrameRefs):
            n, ptrs, pitches = inputs.n, inputs.ptrs, inputs.pitches
        else:
            n = len(inputs)
            ptrs = (_VP * n)(*[t.data_ptr() for t in inputs])
            pitches = (C.c_size_t * n)(*[t.stride(0) for t in inputs])
        _check(_lib.octvr_fastmapper_stitch_nv12(self._h, ptrs, pitches, C.c_void_p(output.data_ptr()), output.stride(0),
                                                 _stream_ptr(stream)))

    def traffic_parts(self):
        """(entry bytes read once per launch, bytes per frame) of one stitch (octvr_fastmapper_traffic_parts)."""
        a, b = C.c_double(), C.c_double()
        _check(_lib.octvr_fastmapper_traffic_parts(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def stitch_nv12_batch(self, frame_sets, outputs=None, stream=None):
        """len(frame_sets) (1, 2 or 4) frames in one launch per plane (octvr_fastmapper_stitch_nv12_batch); outputs:
        one tensor per frame (same pitch).  frame_sets may be a BatchRefs (outputs then None)."""
        b = frame_sets if isinstance(frame_sets, BatchRefs) else BatchRefs(frame_sets, outputs)
        _check(_lib.octvr_fastmapper_stitch_nv12_batch(self._h, b.nf, b.ptrs, b.pitches, b.outs, b.out_pitch,
                                                       _stream_ptr(stream)))

    def close(self):
        if self._h and self._h.value:
            _lib.octvr_fastmapper_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AsyncMultiMapper:
    """vr::AsyncMultiMapper (modules/octvr/src/async.cpp): host YUV420P planes in, host planes out, through
    a 3-deep pinned-buffer pipeline (copy-in, H2D, stitch, D2H, copy-out overlap across frames).

    templates: list of MapperTemplate (all with the same inputs); output_regions: list of (x, y, w, h)
    fractions of out_size; gain_modes[i]: -1 no gain, i estimate, j < i reuse mapper j's gains.
    preview_size (w, h): AsyncMultiMapper::New's preview — each mapper also writes its region of one RGB
    preview image every frame (async.cpp:73-110); read the latest with preview(), or receive every one
    through set_preview_sink()."""

    def __init__(self, templates, in_sizes, out_size, blend_modes, gain_modes, output_regions, device=0, remap="remap",
                 preview_size=(0, 0)):
        if remap not in ("remap", "texture"):
            raise ValueError("remap must be 'remap' or 'texture'")
        self._h = C.c_void_p(0)
        k, n = len(templates), len(in_sizes)
        rigs = (_VP * k)(*[t._h.value for t in templates])
        w = (C.c_int * n)(*[s[0] for s in in_sizes])
        h = (C.c_int * n)(*[s[1] for s in in_sizes])
        bm = (C.c_int * k)(*blend_modes)
        gm = (C.c_int * k)(*gain_modes)
        rg = (C.c_double * (4 * k))(*[float(v) for r in output_regions for v in r])
        hd = _VP()
        pw, ph = (int(v) for v in preview_size)
        if pw or ph:
            _check(_lib.octvr_async_create_preview(rigs, k, device, n, w, h, out_size[0], out_size[1], bm, gm, rg,
                                                   REMAP_TEXTURE if remap == "texture" else 0, pw, ph, C.byref(hd)))
        elif remap == "texture":
            _check(_lib.octvr_async_create_ex(rigs, k, device, n, w, h, out_size[0], out_size[1], bm, gm, rg,
                                              REMAP_TEXTURE, C.byref(hd)))
        else:
            _check(_lib.octvr_async_create(rigs, k, device, n, w, h, out_size[0], out_size[1], bm, gm, rg, C.byref(hd)))
        self._h = hd
        self.preview_size = (pw, ph) if pw * ph > 0 else (0, 0)
        self._sink = None
        self._registered = []
        self._templates = list(templates)  # the mappers copy what they need; kept for symmetry with the reference
        self.n = n
        self.out_size = tuple(out_size)
        self._inflight = []

    def push(self, inputs, output):
        """inputs: list of (Y, U, V) uint8 numpy planes per camera; output: (Y, U, V) planes of the merged
        frame.  The arrays are kept alive until the matching pop()."""
        planes = [p if p.strides[1] == 1 else np.ascontiguousarray(p) for tri in inputs for p in tri]
        for p in list(planes) + list(output):
            assert p.dtype == np.uint8 and p.ndim == 2 and p.strides[1] == 1, "uint8 2-D planes with unit column stride"
        ip = (_VP * len(planes))(*[p.ctypes.data for p in planes])
        ipt = (C.c_size_t * len(planes))(*[p.strides[0] for p in planes])
        op = (_VP * 3)(*[p.ctypes.data for p in output])
        opt = (C.c_size_t * 3)(*[p.strides[0] for p in output])
        _check(_lib.octvr_async_push(self._h, ip, ipt, op, opt))
        self._inflight.append((planes, output))

    def pop(self):
        """Blocks until the oldest pushed frame is written; returns its output planes."""
        rc = _lib.octvr_async_pop(self._h)
        output = self._inflight.pop(0)[1] if self._inflight else None
        _check(rc)
        return output

    def pending(self):
        n = C.c_int()
        _check(_lib.octvr_async_pending(self._h, C.byref(n)))
        return n.value

    def register_output(self, output):
        """Page-lock an output (Y, U, V) plane set the caller will push again (octvr_async_register_output): its
        frames are then downloaded straight into it.  The arrays are kept alive until close()."""
        for p in output:
            assert p.dtype == np.uint8 and p.ndim == 2 and p.strides[1] == 1
        op = (_VP * 3)(*[p.ctypes.data for p in output])
        opt = (C.c_size_t * 3)(*[p.strides[0] for p in output])
        _check(_lib.octvr_async_register_output(self._h, op, opt))
        self._registered.append(tuple(output))

    def unregister_output(self, output):
        op = (_VP * 3)(*[p.ctypes.data for p in output])
        _check(_lib.octvr_async_unregister_output(self._h, op))
        self._registered = [r for r in self._registered if not all(a is b for a, b in zip(r, output))]

    def preview(self):
        """(rgb, header): the latest published preview as an (h, w, 3) uint8 array and its PreviewDataHeader
        (width 0 and rgb None before the first frame completes)."""
        pw, ph = self.preview_size
        rgb = np.zeros((max(ph, 1), max(pw, 1), 3), np.uint8)
        hdr = PreviewDataHeader()
        _check(_lib.octvr_async_pop_preview(self._h, rgb.ctypes.data, rgb.strides[0], C.byref(hdr)))
        return (rgb if hdr.width else None), hdr

    def set_preview_sink(self, fn):
        """fn(rgb, header) on the pipeline's copy-out thread for every frame's preview (rgb: a copy); None
        removes it."""
        if fn is None:
            _check(_lib.octvr_async_set_preview_sink(self._h, PREVIEW_SINK(), None))
            self._sink = None
            return
        pw, ph = self.preview_size

        def _cb(user, p, pitch, hdr):
            a = np.ctypeslib.as_array(p, shape=(ph * pitch,)).reshape(ph, pitch)[:, :pw * 3].reshape(ph, pw, 3).copy()
            h = hdr.contents
            fn(a, PreviewDataHeader(h.width, h.height, h.step, h.fps))

        cb = PREVIEW_SINK(_cb)
        _check(_lib.octvr_async_set_preview_sink(self._h, cb, None))
        self._sink = cb  # keep the ctypes thunk alive

    def info(self):
        """Build-time facts of the pipeline (octvr_async_info): packed_bytes uploaded per frame, runs, ..."""
        buf = C.create_string_buffer(1024)
        _check(_lib.octvr_async_info(self._h, buf, len(buf)))
        import json as _json
        return _json.loads(buf.value.decode())

    def close(self):
        if self._h and self._h.value:
            _lib.octvr_async_destroy(self._h)
            self._h = C.c_void_p(0)
            self._inflight = []
            self._registered = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_lib.octvr_selftest_sat_u8.argtypes = [_VP, _VP, C.c_int, C.c_int, _VP]


def selftest_sat_u8(values, method, stream=None):
    """Device float -> u8 saturating conversion (kernel self-test)."""
    x = values if isinstance(values, torch.Tensor) else torch.tensor(values, dtype=torch.float32)
    x = x.to(device="cuda", dtype=torch.float32).contiguous()
    out = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
    _check(_lib.octvr_selftest_sat_u8(C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), x.numel(), method,
                                      _stream_ptr(stream)))
    return out


def remap_u8(src, map1, map2, scale_x, scale_y, out=None, stream=None):
    """cv::remap INTER_LINEAR on cuda uint8 tensors (H x W [x cn]); maps are cuda float32 (mh x mw)."""
    cn = 1 if src.dim() == 2 else src.shape[2]
    mh, mw = map1.shape
    if out is None:
        out = torch.empty((mh, mw) if cn == 1 else (mh, mw, cn), dtype=torch.uint8, device=src.device)
    _check(_lib.octvr_remap_u8(C.c_void_p(src.data_ptr()), src.shape[1], src.shape[0], src.stride(0), cn,
                               C.c_void_p(map1.data_ptr()), C.c_void_p(map2.data_ptr()), mw, mh, map1.stride(0),
                               scale_x, scale_y, C.c_void_p(out.data_ptr()), out.stride(0), _stream_ptr(stream)))
    return out


def fill_poly(img, pts, color):
    """cv::fillPoly(img, {pts}, color) on a 2-D uint8 numpy array, in place (octvr_fill_poly_u8)."""
    import numpy as np
    assert img.dtype == np.uint8 and img.ndim == 2 and img.flags.c_contiguous
    flat = np.ascontiguousarray(np.asarray(pts, np.int32).reshape(-1))
    _check(_lib.octvr_fill_poly_u8(img.ctypes.data, img.shape[1], img.shape[0],
                                   flat.ctypes.data_as(C.POINTER(C.c_int)), len(flat) // 2, color))
    return img


def png_decode_rgb(data):
    """cv::imdecode(png, IMREAD_COLOR) with the channels in R,G,B order (octvr_png_decode_rgb)."""
    import numpy as np
    w, h = C.c_int(), C.c_int()
    _check(_lib.octvr_png_decode_rgb(data, len(data), None, 0, C.byref(w), C.byref(h)))
    out = np.empty((h.value, w.value, 3), np.uint8)
    _check(_lib.octvr_png_decode_rgb(data, len(data), out.ctypes.data, out.nbytes, C.byref(w), C.byref(h)))
    return out
