"""ctypes binding of include/vmatting.h (libvmatting.so, built in-tree for gfx950).

torch is imported first on purpose: its bundled libamdhip64.so.7 is then the HIP
runtime the library resolves against (same soname), so device pointers and
streams from torch are valid inside every vm_* call.

There is no CPU fallback anywhere in the product: if the library is missing or
no GPU is visible, calls raise.
"""

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
# VM_LIB_PATH: an alternative build of the same library (same-box A/B timing runs); never a fallback
LIB_PATH = os.environ.get("VM_LIB_PATH") or os.path.join(HERE, "libvmatting.so")

VM_F32, VM_BF16, VM_U8, VM_F64, VM_F16 = 0, 1, 2, 3, 4
ACT = {"none": 0, "relu": 1, "sigmoid": 2, "softmax": 3}
VM_OK, VM_EINVAL, VM_EUNSUPPORTED, VM_EHIP, VM_EINDEX = 0, -1, -2, -3, -4
ABI_VERSION = 1

c_void_p, c_int, c_float, c_long, c_size_t = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long, ctypes.c_size_t


class VmTensor(ctypes.Structure):
    _fields_ = [("ptr", c_void_p), ("n", ctypes.c_int32), ("h", ctypes.c_int32), ("w", ctypes.c_int32),
                ("c", ctypes.c_int32), ("cstride", ctypes.c_int32), ("coff", ctypes.c_int32),
                ("dtype", ctypes.c_int32)]


P = ctypes.POINTER(VmTensor)


class VmCropAxis(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("off", ctypes.c_int32), ("lo", ctypes.c_int32), ("hi", ctypes.c_int32),
                ("shift", ctypes.c_int32)]


class VmLoaderSample(ctypes.Structure):
    _fields_ = [("fg", c_void_p), ("prev", c_void_p), ("flow", c_void_p), ("bg", c_void_p),
                ("fg_h", ctypes.c_int32), ("fg_w", ctypes.c_int32), ("prev_h", ctypes.c_int32),
                ("prev_w", ctypes.c_int32), ("bg_h", ctypes.c_int32), ("bg_w", ctypes.c_int32),
                ("fg_rows", VmCropAxis), ("fg_cols", VmCropAxis), ("bg_rows", VmCropAxis), ("bg_cols", VmCropAxis),
                ("mirror", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class VmLoaderOutputs(ctypes.Structure):
    _fields_ = [("ptr", c_void_p * 5), ("pixstride", ctypes.c_int32 * 5), ("reserved", ctypes.c_int32)]


class VmPackJob(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("packed", c_void_p), ("cin", ctypes.c_int32), ("cout", ctypes.c_int32),
                ("dtype", ctypes.c_int32), ("flip", ctypes.c_int32), ("w_cin", ctypes.c_int32),
                ("w_cout", ctypes.c_int32)]


class VmTpsMap(ctypes.Structure):
    _fields_ = [("grid", c_void_p), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("upsample", ctypes.c_int32),
                ("x_span", ctypes.c_int32), ("y_span", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("x_steps", ctypes.c_double), ("y_steps", ctypes.c_double)]


class VmAugmentJob(ctypes.Structure):
    _fields_ = [("fg", c_void_p), ("bg", c_void_p), ("alpha", c_void_p), ("tps_points", c_void_p),
                ("tps_coeffs", c_void_p), ("scratch", c_void_p), ("new_fg", c_void_p), ("new_bg", c_void_p),
                ("new_alpha", c_void_p), ("new_bgra", c_void_p), ("h", ctypes.c_int32), ("w", ctypes.c_int32), ("bg_h", ctypes.c_int32),
                ("bg_w", ctypes.c_int32), ("npts", ctypes.c_int32), ("tu_bg", ctypes.c_int32),
                ("tv_bg", ctypes.c_int32), ("tu_fg", ctypes.c_int32), ("tv_fg", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("m_bg", ctypes.c_double * 6), ("m_fg", ctypes.c_double * 6),
                ("lut", ctypes.c_uint8 * 256)]


LOADER_PLANES = {"cmp": 0, "bg": 1, "label": 2, "warped": 3, "fg": 4}

# (name, restype, argtypes) — one row per declaration in include/vmatting.h
SIGNATURES = [
    ("vm_abi_version", c_int, []),
    ("vm_last_error", ctypes.c_char_p, []),
    ("vm_set_option", c_int, [ctypes.c_char_p, c_long]),
    ("vm_conv3x3_last_kernel", ctypes.c_char_p, []),
    ("vm_conv3x3_packed_bytes", c_size_t, [c_int, c_int, c_int]),
    ("vm_conv3x3_pack_weights", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("vm_conv3x3_nhwc", c_int, [P, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, P, c_void_p]),
    ("vm_conv3x3_pool_nhwc", c_int, [P, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, P, P,
                                     c_void_p]),
    ("vm_conv3x3_head_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, P, c_void_p,
                                     c_void_p]),
    ("vm_conv3x3_head_acc_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, P, c_void_p, c_void_p]),
    ("vm_conv3x3_head_acc_ex_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, P, c_void_p,
                                            c_void_p]),
    ("vm_conv3x3_pair_first_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                           c_void_p, c_int, P, P, c_void_p]),
    ("vm_conv3x3_pair_first_mid_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                               c_void_p, c_int, P, P, P, c_void_p]),
    ("vm_conv3x3_pair_first_head_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                                c_void_p, c_int, P, P, c_void_p, c_int, c_int, c_void_p, c_int,
                                                c_void_p]),
    ("vm_conv3x3_head_partial_nhwc", c_int, [P, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, P, c_void_p,
                                             c_void_p, c_void_p]),
    ("vm_conv3x3_fold_up2x_weights", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("vm_conv3x3_up2x_nhwc", c_int, [P, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, P,
                                     c_void_p]),
    ("vm_conv3x3_up2x_head_nhwc", c_int, [P, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                          P, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    ("vm_conv3x3_head_from_partials", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, P, c_void_p,
                                              c_void_p]),
    ("vm_maxpool2x2_same_nhwc", c_int, [P, P, c_void_p]),
    ("vm_resize_bilinear_tf1_nhwc", c_int, [P, P, c_void_p]),
    ("vm_convert_nhwc", c_int, [P, P, c_void_p, c_void_p, c_int, c_void_p]),
    ("vm_stream_create_masked", c_int, [ctypes.POINTER(c_void_p)]),
    ("vm_stream_destroy", c_int, [c_void_p]),
    ("vm_spin", c_int, [c_int, c_void_p]),
    ("vm_split6_nhwc", c_int, [P, P, P, c_void_p]),
    ("vm_split3h_nhwc", c_int, [P, P, P, c_int, c_void_p, c_void_p]),
    ("vm_resize_split3h_nhwc", c_int, [P, P, c_int, c_void_p, c_void_p]),
    ("vm_conv3x3_up2x_split3_nhwc", c_int, [P, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                            P, c_int, c_void_p, c_void_p]),
    ("vm_conv3x3_split3_nhwc", c_int, [P, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, P, c_int, P,
                                       c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    ("vm_bn_workspace_bytes", c_size_t, [P]),
    ("vm_bn_stats_nhwc", c_int, [P, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("vm_bn_apply_nhwc", c_int, [P, P, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p]),
    ("vm_softmax_lastdim_nhwc", c_int, [P, P, c_void_p]),
    ("vm_composite_image", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_long, c_int, c_void_p, c_int,
                                   c_void_p]),
    ("vm_remap_bilinear_f32", c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                      c_void_p]),
    ("vm_remap_bilinear_u8", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("vm_fb_consistency", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_float, c_int, c_void_p, c_void_p]),
    ("vm_temporal_refine_input", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                                         c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    ("vm_loss_workspace_bytes", c_size_t, [c_long]),
    ("vm_matting_loss", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p,
                                c_void_p]),
    ("vm_loader_workspace_bytes", c_size_t, [c_int]),
    ("vm_loader_compose", c_int, [ctypes.POINTER(VmLoaderSample), c_int, c_int, c_int, c_int,
                                  ctypes.POINTER(VmLoaderOutputs), c_void_p, c_void_p]),
    ("vm_tps_grid", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.c_double, ctypes.c_double,
                            ctypes.c_double, ctypes.c_double, c_void_p, c_void_p]),
    ("vm_tps_sample", c_int, [ctypes.POINTER(VmTpsMap), c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p]),
    ("vm_warp_affine", c_int, [c_void_p, c_int, c_int, c_int, c_int, ctypes.POINTER(ctypes.c_double), c_void_p,
                               c_int, c_int, c_void_p]),
    ("vm_warp_image", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(ctypes.c_uint8), c_void_p, c_int, c_int, c_void_p]),
    ("vm_change_illumination_u8", c_int, [c_void_p, c_long, ctypes.POINTER(ctypes.c_uint8), c_void_p, c_void_p]),
    ("vm_nonzero_stats", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("vm_bgra_u8", c_int, [c_void_p, c_void_p, c_int, c_long, c_void_p, c_void_p]),
    ("vm_augment_scratch_bytes", ctypes.c_size_t, [c_int, c_int]),
    ("vm_bgra_u8_batch", c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), ctypes.POINTER(c_long),
                                 ctypes.POINTER(c_void_p), c_int, c_void_p]),
    ("vm_augment_batch", c_int, [ctypes.POINTER(VmAugmentJob), c_int, c_void_p]),
    ("vm_nonzero_stats_batch", c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int,
                                       c_void_p, c_void_p]),
    ("vm_trimap_from_matte", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("vm_matting_loss_backward", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                                         c_void_p]),
    ("vm_bn_backward_workspace_bytes", c_size_t, [c_int]),
    ("vm_bn_backward_nhwc", c_int, [P, P, P, c_void_p, c_void_p, c_void_p, c_float, P, c_void_p, c_void_p, c_void_p,
                                    c_void_p]),
    ("vm_bn_backward_ex_nhwc", c_int, [P, P, P, c_void_p, c_void_p, c_void_p, c_float, P, P, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    ("vm_bn_backward_apply_nhwc", c_int, [P, P, P, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_long,
                                          P, P, c_void_p]),
    ("vm_relu_backward_nhwc", c_int, [P, P, P, c_void_p]),
    ("vm_relu_backward_ex_nhwc", c_int, [P, P, P, P, c_void_p]),
    ("vm_relu_backward_split_nhwc", c_int, [P, P, c_int, P, P, P, c_void_p]),
    ("vm_maxpool2x2_backward_nhwc", c_int, [P, P, P, P, c_void_p]),
    ("vm_relu_backward_bias_workspace_bytes", c_size_t, [c_int]),
    ("vm_relu_backward_bias_nhwc", c_int, [P, P, P, P, c_void_p, c_void_p, c_void_p]),
    ("vm_resize_bilinear_tf1_backward", c_int, [P, c_void_p, c_int, c_int, c_void_p]),
    ("vm_resize_bilinear_tf1_backward_nhwc", c_int, [P, P, c_void_p]),
    ("vm_conv3x3_wgrad_workspace_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    ("vm_conv3x3_wgrad_nhwc", c_int, [P, P, c_void_p, c_void_p, c_void_p]),
    ("vm_conv3x3_workspace_bytes", c_size_t, [P, c_int, c_int]),
    ("vm_conv3x3_ex_nhwc", c_int, [P, c_int, c_long, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, P,
                                   c_void_p, c_size_t, c_void_p]),
    ("vm_conv3x3_pack_weights_batch", c_int, [c_int, ctypes.POINTER(VmPackJob), c_void_p]),
    ("vm_conv3x3_sources_nhwc", c_int, [P, c_int, c_long, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                        c_int, P, c_void_p]),
    ("vm_conv3x3_wgrad_ex_workspace_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    ("vm_conv3x3_wgrad_ex_nhwc", c_int, [P, c_int, c_long, P, c_void_p, c_void_p, c_int, c_void_p]),
    ("vm_conv3x3_flip_weights", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("vm_adam_tf", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_float, c_float, c_float, c_float,
                           c_float, c_void_p]),
]

_lib = None


def lib():
    """Load libvmatting.so once; raise (never fall back) if it is absent or stale."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("vmatting: %s not built — run `make -C video-matting_amd` or "
                               "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
        l = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if not hasattr(l, name) and os.environ.get("VM_LIB_PATH"):
                continue  # an A/B build of an older tree: entry points added since are simply absent
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        if l.vm_abi_version() != ABI_VERSION:
            raise RuntimeError("vmatting: ABI %d != %d, rebuild the library" % (l.vm_abi_version(), ABI_VERSION))
        _lib = l
    return _lib


def check(rc, what):
    if rc == VM_OK:
        return
    msg = "%s: %s" % (what, lib().vm_last_error().decode(errors="replace"))
    if rc == VM_EINVAL:
        raise ValueError(msg)
    if rc == VM_EINDEX:
        raise IndexError(msg)
    if rc == VM_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def set_option(key, value):
    """vm_set_option: process-wide kernel-selection knobs ("conv_kernel", "conv_min_tiles")."""
    check(lib().vm_set_option(key.encode(), int(value)), "set_option")


def last_conv_kernel():
    """vm_conv3x3_last_kernel: rocprofv3 spelling of the kernel the last conv call launched."""
    return lib().vm_conv3x3_last_kernel().decode()


# torch's private C getters behind torch.cuda.current_stream(d).cuda_stream, looked up once; if a torch release
# renames or drops them, current_raw_stream falls back to the public call (same handle, ~6 us more per launch)
_GET_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def current_raw_stream(device_index=None):
    """The current stream's raw hipStream_t (as an int) on ``device_index`` (default: the current device).  The same
    handle as torch.cuda.current_stream(d).cuda_stream, from the two C-level getters that call wraps: that call
    builds a Stream object and resolves the device through several Python layers, ~6 us per call, and every
    kernel launch asks for it (profiled: ~230 calls = ~1.4 ms of host time per training step)."""
    if _GET_RAW_STREAM is None or _GET_DEVICE is None:
        return torch.cuda.current_stream(device_index).cuda_stream
    if not torch.cuda.is_initialized():
        torch.cuda.init()
    return _GET_RAW_STREAM(_GET_DEVICE() if device_index is None else device_index)


def stream_handle(stream=None):
    return c_void_p(current_raw_stream() if stream is None else stream.cuda_stream)
