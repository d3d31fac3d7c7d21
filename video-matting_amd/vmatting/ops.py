"""Tensor-level wrappers over the C ABI (torch tensors on a ROCm device in, out).

Each function is one TF/OpenCV op of the reference (cited in include/vmatting.h).
NHWC views: any torch tensor whose last dim is contiguous and whose pixel rows
are evenly strided (stride(1) == W*stride(2), stride(0) == H*stride(1)) — in
particular a channel slice ``buf[..., a:b]`` of a wider buffer, which is how
tf.concat is expressed without copies.
"""

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import VmTensor, check, lib, stream_handle

_DT = {torch.float32: _lib.VM_F32, torch.bfloat16: _lib.VM_BF16, torch.uint8: _lib.VM_U8,
       torch.float16: _lib.VM_F16}  # (fp16: the split-fp16 x3 conv operands only, vmatting/split3.py)
TORCH_DTYPE = {"fp32": torch.float32, "f32": torch.float32, "float32": torch.float32,
               "bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "f16": torch.float16}


def _require_gpu(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise TypeError("vmatting ops take ROCm device tensors (got %r)" % (type(t) if not isinstance(t, torch.Tensor)
                                                                          else t.device))


def nhwc(t):
    """Describe a 4-D NHWC torch view as a vm_tensor (by value)."""
    _require_gpu(t)
    if t.dim() != 4:
        raise ValueError("expected NHWC 4-D tensor, got shape %s" % (tuple(t.shape),))
    n, h, w, c = t.shape
    s0, s1, s2, s3 = t.stride()
    if s3 != 1 or (h > 1 and s1 != w * s2) or (n > 1 and s0 != h * s1):
        raise ValueError("tensor is not an NHWC channel-slice view (strides %s)" % (t.stride(),))
    if t.dtype not in _DT:
        raise TypeError("unsupported dtype %s" % t.dtype)
    return VmTensor(t.data_ptr(), n, h, w, c, s2, 0, _DT[t.dtype])


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _f32(t):
    if t is None:
        return None
    _require_gpu(t)
    assert t.dtype == torch.float32 and t.is_contiguous()
    return t


# ---------------------------------------------------------------------------------------------- conv

class PackedConv:
    """One 3x3 conv's weights in kernel layout, plus its f32 bias / per-channel affine (folded BN).

    ``w_hwio``: TF-layout filter [3,3,cin,cout] (numpy or tensor).  The reference creates
    these in unet.py:11-17 (init_conv) / 65-74 (VGG filters).
    """

    def __init__(self, w_hwio, bias=None, dtype="bf16", device="cuda", scale=None, shift=None):
        w = torch.as_tensor(np.asarray(w_hwio, np.float32) if not isinstance(w_hwio, torch.Tensor) else w_hwio,
                            dtype=torch.float32).to(device).contiguous()
        if w.dim() != 4 or w.shape[0] != 3 or w.shape[1] != 3:
            raise ValueError("expected a [3,3,cin,cout] filter, got %s" % (tuple(w.shape),))
        self.cin, self.cout = int(w.shape[2]), int(w.shape[3])
        self.dtype = TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.w_hwio = w
        vdt = _DT[self.dtype]
        nbytes = lib().vm_conv3x3_packed_bytes(self.cin, self.cout, vdt)
        self.packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
        check(lib().vm_conv3x3_pack_weights(_ptr(w), self.cin, self.cout, vdt, _ptr(self.packed),
                                            stream_handle()), "pack_weights")
        as_f = lambda v: None if v is None else torch.as_tensor(np.asarray(v, np.float32) if not isinstance(  # noqa
            v, torch.Tensor) else v, dtype=torch.float32).to(device).contiguous()
        self.bias = as_f(bias)
        self.scale = as_f(scale)
        self.shift = as_f(shift)

    @classmethod
    def from_source(cls, src, cin, cout, dtype="bf16", flip=False, bias=None):
        """A (cin, cout) conv packed from the f32 HWIO filter ``src`` with zeros outside it: a cout-padded copy of a
        narrow conv (flip=False), or the data-gradient conv of ``src`` (flip=True: spatially flipped, in/out
        transposed, so cin >= src's cout and cout = src's cin).  ``src`` is read again by every pack_batch."""
        self = cls.__new__(cls)
        self.cin, self.cout = int(cin), int(cout)
        self.dtype = TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.w_hwio, self._src, self._flip = None, src, bool(flip)  # src: a tensor, or a PackedConv (its filter)
        nbytes = lib().vm_conv3x3_packed_bytes(self.cin, self.cout, _DT[self.dtype])
        self.packed = torch.empty(nbytes, dtype=torch.uint8, device=self._source().device)
        self.bias, self.scale, self.shift = bias, None, None
        pack_batch([self])
        return self

    def _source(self):
        src = self.w_hwio if self.w_hwio is not None else self._src
        return src.w_hwio if isinstance(src, PackedConv) else src

    def pack_job(self):
        src = self._source()
        flip = getattr(self, "_flip", False)
        return _lib.VmPackJob(_ptr(src), _ptr(self.packed), self.cin, self.cout, _DT[self.dtype], int(flip),
                              int(src.shape[2]), int(src.shape[3]))

    def up2x(self):
        """The folded-resize weights of this filter (vm_conv3x3_fold_up2x_weights + pack, cout' = 4*cout),
        built once on first use; None when the compute dtype has no folded path (f32)."""
        if self.dtype != torch.bfloat16 or self.cout % 64:
            return None
        if getattr(self, "_up", None) is None:
            dev = self.packed.device
            wu = torch.empty((3, 3, self.cin, 4 * self.cout), dtype=torch.float32, device=dev)
            check(lib().vm_conv3x3_fold_up2x_weights(_ptr(self.w_hwio), self.cin, self.cout, _ptr(wu),
                                                     stream_handle()), "fold_up2x_weights")
            nbytes = lib().vm_conv3x3_packed_bytes(self.cin, 4 * self.cout, _DT[self.dtype])
            self._up = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            check(lib().vm_conv3x3_pack_weights(_ptr(wu), self.cin, 4 * self.cout, _DT[self.dtype], _ptr(self._up),
                                                stream_handle()), "pack_weights(up2x)")
        return self._up

    def repack(self):
        """Re-pack after the f32 HWIO filter changed in place (the optimizer step of train.VideoTrainer)."""
        pack_batch([self])
        return self

    def set_affine(self, scale, shift):
        self.scale = None if scale is None else torch.as_tensor(scale, dtype=torch.float32).to(self.packed.device)
        self.shift = None if shift is None else torch.as_tensor(shift, dtype=torch.float32).to(self.packed.device)

    def __call__(self, x, act="none", out=None, out_dtype=None, affine=None):
        return conv3x3(x, self, act, out, out_dtype, affine)


class PackBatch:
    """Re-pack many PackedConvs in one launch (vm_conv3x3_pack_weights_batch); the job array is built once, so the
    sources and packed buffers must stay where they are (the trainer's flat parameter buffer does)."""

    def __init__(self, convs):
        self.convs = list(convs)
        self.jobs = (_lib.VmPackJob * max(1, len(self.convs)))(*[pc.pack_job() for pc in self.convs])

    def __call__(self):
        check(lib().vm_conv3x3_pack_weights_batch(len(self.convs), self.jobs, stream_handle()), "pack_weights_batch")
        for pc in self.convs:
            pc._up = None


def pack_batch(convs):
    PackBatch(convs)()


class SourceConcat:
    """The channel concat of ``nsrc`` equally shaped feature maps stored one after another in ``base``
    ([nsrc*N, H, W, C], contiguous) — unet_simple.py:153-168's per-level concat of the three VGG towers, which
    run as ONE batch-3N pass here.  Never materialised: conv3x3 / conv_wgrad read it as split sources."""

    def __init__(self, base, nsrc):
        if base.dim() != 4 or base.shape[0] % nsrc or not base.is_contiguous():
            raise ValueError("SourceConcat: base must be a contiguous [nsrc*N,H,W,C] tensor")
        self.base, self.nsrc = base, int(nsrc)
        n = base.shape[0] // nsrc
        self.src0 = base[:n]
        self.stride = n * base.shape[1] * base.shape[2] * base.shape[3]
        self.shape = (n, base.shape[1], base.shape[2], nsrc * base.shape[3])
        self.dtype, self.device, self.is_cuda = base.dtype, base.device, base.is_cuda

    def source(self, i):
        n = self.shape[0]
        return self.base[i * n:(i + 1) * n]

    def materialize(self):
        return torch.cat([self.source(i) for i in range(self.nsrc)], -1)


def conv3x3(x, pc, act="none", out=None, out_dtype=None, affine=None, pool_out=None, splitk=False):
    """tf.nn.conv2d 3x3 SAME + bias_add (+ folded BN affine) + activation, on MFMA.

    ``affine``: None -> the PackedConv's own scale/shift; False -> none; (scale, shift) -> those.
    ``pool_out``: also write tf.nn.max_pool 2x2/2 SAME of the result there (fused into the conv epilogue when
    the kernel supports it, else a separate max-pool launch).
    ``splitk``: allow split-K on small grids (a workspace is passed; the per-pixel summation order then depends
    on the batch size, so the inference nets, whose frames must not depend on their batch, leave it off).
    """
    if x.dtype != pc.dtype:
        raise TypeError("conv input dtype %s != packed weights dtype %s" % (x.dtype, pc.dtype))
    if x.shape[-1] != pc.cin:
        raise ValueError("conv input has %d channels, filter expects %d" % (x.shape[-1], pc.cin))
    n, h, w, _ = x.shape
    if out is None:
        out = torch.empty((n, h, w, pc.cout), dtype=out_dtype or x.dtype, device=x.device)
    if affine is None:
        scale, shift = pc.scale, pc.shift
    elif affine is False:
        scale = shift = None
    else:
        scale, shift = affine
    if isinstance(x, SourceConcat) or pool_out is None:
        # the general entry: split sources and/or a workspace for split-K on small grids
        if isinstance(x, SourceConcat):
            xv, nsrc, stride = nhwc(x.src0), x.nsrc, x.stride
            if pool_out is not None:
                raise ValueError("conv3x3: no fused pooling over split sources")
        else:
            xv, nsrc, stride = nhwc(x), 1, 0
        yv = nhwc(out)
        wsz = lib().vm_conv3x3_workspace_bytes(ctypes.byref(xv), pc.cin, pc.cout) if splitk else 0
        ws = _workspace(wsz, x.device) if wsz else None
        prof = _CONV_PROFILE
        if prof is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        rc = lib().vm_conv3x3_ex_nhwc(ctypes.byref(xv), nsrc, stride, _ptr(pc.packed), pc.cin, pc.cout,
                                      _ptr(pc.bias), _ptr(scale), _ptr(shift), _lib.ACT[act], ctypes.byref(yv),
                                      _ptr(ws), wsz, stream_handle())
        if rc == _lib.VM_EUNSUPPORTED and nsrc > 1:
            # sources spread wider than the kernels' 32-bit offsets reach (large batches): one materialised concat
            xm = x.materialize()
            xv = nhwc(xm)
            rc = lib().vm_conv3x3_ex_nhwc(ctypes.byref(xv), 1, 0, _ptr(pc.packed), pc.cin, pc.cout, _ptr(pc.bias),
                                          _ptr(scale), _ptr(shift), _lib.ACT[act], ctypes.byref(yv), _ptr(ws), wsz,
                                          stream_handle())
        check(rc, "conv3x3")
        if prof is not None:
            ev1.record()
            prof.append((2 * n * h * w * 9 * pc.cin * pc.cout, _lib.last_conv_kernel(), ev0, ev1,
                         (n, h, w, pc.cin, pc.cout)))
        return out
    xv, yv = nhwc(x), nhwc(out)
    prof = _CONV_PROFILE
    if prof is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    fused = False
    if pool_out is not None:
        pv = nhwc(pool_out)
        rc = lib().vm_conv3x3_pool_nhwc(ctypes.byref(xv), _ptr(pc.packed), pc.cin, pc.cout, _ptr(pc.bias),
                                        _ptr(scale), _ptr(shift), _lib.ACT[act], ctypes.byref(yv), ctypes.byref(pv),
                                        stream_handle())
        if rc != _lib.VM_EUNSUPPORTED:
            check(rc, "conv3x3_pool")
            fused = True
    if not fused:
        check(lib().vm_conv3x3_nhwc(ctypes.byref(xv), _ptr(pc.packed), pc.cin, pc.cout, _ptr(pc.bias), _ptr(scale),
                                    _ptr(shift), _lib.ACT[act], ctypes.byref(yv), stream_handle()), "conv3x3")
    if prof is not None:
        ev1.record()
        prof.append((2 * n * h * w * 9 * pc.cin * pc.cout, _lib.last_conv_kernel(), ev0, ev1,
                     (n, h, w, pc.cin, pc.cout)))
    if pool_out is not None and not fused:
        maxpool2x2(out, out=pool_out)
    return out


def conv_head(x, pc, act="none", out=None, alpha=None, partial=None):
    """cout == 1 conv (unet.py:203-204 conv1_5) into ``out``; with ``alpha`` (contiguous f32, one value per pixel)
    also tf.nn.sigmoid of the pre-activation from the same pass (unet.py:205), saving a separate elementwise launch."""
    if pc.cout != 1:
        raise ValueError("conv_head needs a cout == 1 filter")
    if x.dtype != pc.dtype:
        raise TypeError("conv input dtype %s != packed weights dtype %s" % (x.dtype, pc.dtype))
    n, h, w, _ = x.shape
    if out is None:
        out = torch.empty((n, h, w, 1), dtype=torch.float32, device=x.device)
    if alpha is not None:
        _require_gpu(alpha)
        if alpha.dtype != torch.float32 or not alpha.is_contiguous() or alpha.numel() != n * h * w:
            raise ValueError("alpha must be a contiguous f32 tensor of n*h*w elements")
    xv, yv = nhwc(x), nhwc(out)
    prof = _CONV_PROFILE
    if prof is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    if partial is not None:  # + the per-tap shares of the channels x does not carry (conv_pair_first_head)
        if partial.dtype != torch.float32 or not partial.is_contiguous() or tuple(partial.shape) != (n, h, w, 12):
            raise ValueError("partial must be a contiguous f32 [n,h,w,12] tensor")
        check(lib().vm_conv3x3_head_partial_nhwc(ctypes.byref(xv), _ptr(pc.packed), pc.cin, _ptr(pc.bias),
                                                 _ptr(pc.scale), _ptr(pc.shift), _lib.ACT[act], ctypes.byref(yv),
                                                 _ptr(alpha), _ptr(partial), stream_handle()), "conv3x3_head_partial")
    else:
        check(lib().vm_conv3x3_head_nhwc(ctypes.byref(xv), _ptr(pc.packed), pc.cin, _ptr(pc.bias), _ptr(pc.scale),
                                         _ptr(pc.shift), _lib.ACT[act], ctypes.byref(yv), _ptr(alpha),
                                         stream_handle()), "conv3x3_head")
    if prof is not None:
        ev1.record()
        prof.append((2 * n * h * w * 9 * pc.cin, _lib.last_conv_kernel(), ev0, ev1))
    return out


def conv_pair_first_head(x, pc1, pc2, head_w, head_coff, partial, act2="relu", out=None, pool_out=None,
                         store_y=False, fallback=False):
    """conv_pair_first with the head split (vm_conv3x3_pair_first_head_nhwc): besides pool_out (and ``out`` when
    store_y) the pair kernel writes ``partial`` [n,h,w,12] f32 = per-tap shares of the cout == 1 head filter
    ``head_w`` (device f32 HWIO [3,3,cin_head,1]) over its output channels, which sit at head_coff of the head's
    input (unet.py:203: conv1_5 over cat1 = [upconv_4, conv1_2]).  conv_head(..., partial=partial) finishes it.
    ``fallback``: return None instead of raising when the kernel cannot take the case (the caller runs the
    unsplit path)."""
    n, h, w, _ = x.shape
    if pc1.dtype != torch.bfloat16 or pc2.dtype != torch.bfloat16 or pc1.cout != 64 or pc2.cin != 64:
        raise NotImplementedError("conv_pair_first_head: bf16 64-channel pair only")
    if head_w.dtype != torch.float32 or not head_w.is_contiguous() or head_w.dim() != 4 or head_w.shape[3] != 1:
        raise ValueError("head_w must be a contiguous f32 [3,3,cin,1] filter")
    if partial.dtype != torch.float32 or not partial.is_contiguous() or tuple(partial.shape) != (n, h, w, 12):
        raise ValueError("partial must be a contiguous f32 [n,h,w,12] tensor")
    _require_gpu(head_w)
    _require_gpu(partial)
    if out is None:
        out = torch.empty((n, h, w, pc2.cout), dtype=torch.bfloat16, device=x.device)
    xv, yv = nhwc(x), nhwc(out)
    pv = nhwc(pool_out) if pool_out is not None else None
    prof = _CONV_PROFILE
    if prof is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = lib().vm_conv3x3_pair_first_head_nhwc(
        ctypes.byref(xv), _ptr(pc1.packed), pc1.cin, _ptr(pc1.bias), _ptr(pc2.packed), pc2.cout, _ptr(pc2.bias),
        _ptr(pc2.scale), _ptr(pc2.shift), _lib.ACT[act2], ctypes.byref(yv),
        ctypes.byref(pv) if pv is not None else None, _ptr(head_w), int(head_w.shape[2]), head_coff, _ptr(partial),
        int(bool(store_y)), stream_handle())
    if rc == _lib.VM_EUNSUPPORTED and fallback:
        return None  # e.g. a kernel-selection override (vm_set_option "conv_kernel"/"pair_kernel") rules it out
    check(rc, "conv3x3_pair_first_head")
    if prof is not None:
        ev1.record()
        prof.append((2 * n * h * w * 9 * (pc1.cin * pc1.cout + pc2.cin * pc2.cout), _lib.last_conv_kernel(), ev0, ev1))
    return out


def conv_pair_first(x, pc1, pc2, act2="relu", out=None, pool_out=None, mid=None, keep_mid=False):
    """conv3x3(relu(conv3x3(x, pc1)), pc2) (+ 2x2 SAME max-pool into pool_out): unet.py:170-172, conv1_1 -> conv1_2
    (-> pool1).  bf16 runs ONE kernel whose 64-channel intermediate stays in LDS (vm_conv3x3_pair_first_nhwc); any
    other case runs the two convs through ``mid`` (the intermediate, allocated when None).  ``keep_mid``: ``mid``
    receives conv1_1's output in every case (the fused kernel writes it too, vm_conv3x3_pair_first_mid_nhwc)."""
    n, h, w, _ = x.shape
    if out is None:
        out = torch.empty((n, h, w, pc2.cout), dtype=x.dtype, device=x.device)
    if x.dtype in (torch.bfloat16, torch.float32) and pc1.dtype == pc2.dtype == torch.bfloat16 and pc1.cout == 64 \
            and pc2.cin == 64:
        xv, yv = nhwc(x), nhwc(out)
        pv = nhwc(pool_out) if pool_out is not None else None
        prof = _CONV_PROFILE
        if prof is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        if keep_mid:
            if mid is None or mid.dtype != torch.bfloat16:
                raise ValueError("keep_mid needs a bf16 mid buffer")
            mv = nhwc(mid)
            rc = lib().vm_conv3x3_pair_first_mid_nhwc(ctypes.byref(xv), _ptr(pc1.packed), pc1.cin, _ptr(pc1.bias),
                                                      _ptr(pc2.packed), pc2.cout, _ptr(pc2.bias), _ptr(pc2.scale),
                                                      _ptr(pc2.shift), _lib.ACT[act2], ctypes.byref(yv),
                                                      ctypes.byref(pv) if pv is not None else None, ctypes.byref(mv),
                                                      stream_handle())
        else:
            rc = lib().vm_conv3x3_pair_first_nhwc(ctypes.byref(xv), _ptr(pc1.packed), pc1.cin, _ptr(pc1.bias),
                                                  _ptr(pc2.packed), pc2.cout, _ptr(pc2.bias), _ptr(pc2.scale),
                                                  _ptr(pc2.shift), _lib.ACT[act2], ctypes.byref(yv),
                                                  ctypes.byref(pv) if pv is not None else None, stream_handle())
        if rc != _lib.VM_EUNSUPPORTED:
            check(rc, "conv3x3_pair_first")
            if prof is not None:
                ev1.record()
                prof.append((2 * n * h * w * 9 * (pc1.cin * pc1.cout + pc2.cin * pc2.cout), _lib.last_conv_kernel(),
                             ev0, ev1))
            return out
    if x.dtype != pc1.dtype:  # the unfused path takes the frame in the compute dtype, channels padded to 8
        c = x.shape[-1]
        xb = torch.empty((n, h, w, (c + 7) // 8 * 8), dtype=pc1.dtype, device=x.device)
        x = convert(x, xb)[..., :c]
    m = conv3x3(x, pc1, "relu", out=mid)
    return conv3x3(m, pc2, act2, out=out, pool_out=pool_out)


def upconv3x3(x, pc, act="none", out=None, size=None, rbuf=None, fold=True):
    """tf.image.resize_images(x, size) -> conv3x3 (unet.py:44-63, the upconv half of upconv_concat).

    Exact 2x upsampling in bf16 runs as ONE folded conv on the low-res frame (vm_conv3x3_up2x_nhwc, no resized
    tensor in HBM) when ``fold``; any other case is the resize kernel (into ``rbuf`` if given) followed by the
    conv kernel."""
    n, h, w, _ = x.shape
    oh, ow = (2 * h, 2 * w) if size is None else (int(size[0]), int(size[1]))
    if out is None:
        out = torch.empty((n, oh, ow, pc.cout), dtype=x.dtype, device=x.device)
    up = pc.up2x() if fold and (oh, ow) == (2 * h, 2 * w) and x.dtype == pc.dtype else None
    if up is not None:
        xv, yv = nhwc(x), nhwc(out)
        prof = _CONV_PROFILE
        if prof is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        rc = lib().vm_conv3x3_up2x_nhwc(ctypes.byref(xv), _ptr(up), _ptr(pc.packed), pc.cin, pc.cout, _ptr(pc.bias),
                                        _ptr(pc.scale), _ptr(pc.shift), _lib.ACT[act], ctypes.byref(yv),
                                        stream_handle())
        if rc != _lib.VM_EUNSUPPORTED:
            check(rc, "conv3x3_up2x")
            if prof is not None:
                ev1.record()
                prof.append((2 * n * oh * ow * 9 * pc.cin * pc.cout, _lib.last_conv_kernel(), ev0, ev1))
            return out
    r = resize_bilinear(x, (oh, ow), out=rbuf)
    return conv3x3(r, pc, act, out=out)


def upconv3x3_head(x, pc, head_w, head_coff, partial, act="none", out=None, store_y=False):
    """upconv3x3 (exact 2x, folded) with the head split (vm_conv3x3_up2x_head_nhwc): besides ``out`` (written only
    when store_y) the conv writes ``partial`` [n,2h,2w,12] f32 = per-tap shares of the cout == 1 head filter
    ``head_w`` (device f32 HWIO [3,3,cin_head,1]) over its 64 output channels, which sit at head_coff of the head's
    input (unet.py:200-205: conv1_5 over cat1 = [upconv_4, conv1_2]).  Returns None when the kernel cannot take the
    case (the caller runs the unsplit path)."""
    n, h, w, _ = x.shape
    up = pc.up2x() if x.dtype == pc.dtype == torch.bfloat16 and pc.cout == 64 else None
    if up is None:
        return None
    if head_w.dtype != torch.float32 or not head_w.is_contiguous() or head_w.dim() != 4 or head_w.shape[3] != 1:
        raise ValueError("head_w must be a contiguous f32 [3,3,cin,1] filter")
    if partial.dtype != torch.float32 or not partial.is_contiguous() or tuple(partial.shape) != (n, 2 * h, 2 * w, 12):
        raise ValueError("partial must be a contiguous f32 [n,2h,2w,12] tensor")
    _require_gpu(head_w)
    _require_gpu(partial)
    if out is None:
        out = torch.empty((n, 2 * h, 2 * w, pc.cout), dtype=x.dtype, device=x.device)
    xv, yv = nhwc(x), nhwc(out)
    prof = _CONV_PROFILE
    if prof is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = lib().vm_conv3x3_up2x_head_nhwc(
        ctypes.byref(xv), _ptr(up), _ptr(pc.packed), pc.cin, pc.cout, _ptr(pc.bias), _ptr(pc.scale), _ptr(pc.shift),
        _lib.ACT[act], ctypes.byref(yv), _ptr(head_w), int(head_w.shape[2]), head_coff, _ptr(partial),
        int(bool(store_y)), stream_handle())
    if rc == _lib.VM_EUNSUPPORTED:
        return None
    check(rc, "conv3x3_up2x_head")
    if prof is not None:
        ev1.record()
        prof.append((2 * n * 4 * h * w * 9 * pc.cin * pc.cout, _lib.last_conv_kernel(), ev0, ev1))
    return out


def head_from_partials(pa, pb, bias=None, logits=None, alpha=None):
    """conv1_5 + sigmoid from the two halves' per-tap partials (vm_conv3x3_head_from_partials): logits =
    bias + sum_tap (pa + pb)[p + off(tap)][tap], alpha = sigmoid(logits).  pa, pb: contiguous f32 [n,h,w,12]."""
    n, h, w, k = pa.shape
    if k != 12 or tuple(pb.shape) != (n, h, w, 12) or pa.dtype != torch.float32 or pb.dtype != torch.float32 \
            or not pa.is_contiguous() or not pb.is_contiguous():
        raise ValueError("pa, pb must be contiguous f32 [n,h,w,12] partials")
    _require_gpu(pa)
    _require_gpu(pb)
    if logits is None:
        logits = torch.empty((n, h, w, 1), dtype=torch.float32, device=pa.device)
    lv = nhwc(logits)
    if alpha is not None and (alpha.dtype != torch.float32 or not alpha.is_contiguous() or alpha.numel() != n * h * w):
        raise ValueError("alpha must be a contiguous f32 tensor of n*h*w values")
    prof = _CONV_PROFILE
    if prof is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    check(lib().vm_conv3x3_head_from_partials(_ptr(pa), _ptr(pb), n, h, w, _ptr(bias), ctypes.byref(lv),
                                              _ptr(alpha), stream_handle()), "head_from_partials")
    if prof is not None:  # (the head's own conv FLOPs were made in the two epilogues; listed for its time)
        ev1.record()
        prof.append((2 * n * h * w * 9 * 128, _lib.last_conv_kernel(), ev0, ev1))
    return logits


# When a list, conv3x3 appends (algorithmic FLOPs, is_head, start_event, end_event) per launch —
# HIP events on the launch stream, used by bench.py for the roofline's achieved TFLOP/s.
_CONV_PROFILE = None


def conv_profile(enable):
    global _CONV_PROFILE
    _CONV_PROFILE = [] if enable else None
    return _CONV_PROFILE


# ---------------------------------------------------------------------------------------------- memory-bound ops

def maxpool2x2(x, out=None):
    """tf.nn.max_pool 2x2/2 SAME."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, (h + 1) // 2, (w + 1) // 2, c), dtype=x.dtype, device=x.device)
    xv, yv = nhwc(x), nhwc(out)
    check(lib().vm_maxpool2x2_same_nhwc(ctypes.byref(xv), ctypes.byref(yv), stream_handle()), "maxpool2x2")
    return out


def widen(x, c):
    """The channel view ``x`` widened to ``c`` channels over the same storage: the zero pad channels of a padded
    buffer, read by a conv whose pack is channel-padded (UNetSimple.padded).  x's channel stride must cover c."""
    if x.shape[-1] == c:
        return x
    cs = x.stride(-2)
    if x.dim() != 4 or x.stride(-1) != 1 or (x.storage_offset() % cs) + c > cs:
        raise ValueError("widen: a [N,H,W,%d] view needs %d channels of stride, has %d" % (x.shape[-1], c, cs))
    return x.as_strided(tuple(x.shape[:-1]) + (c,), x.stride(), x.storage_offset())


def resize_bilinear(x, size, out=None):
    """tf.image.resize_images(x, size) with TF-1.x defaults (bilinear, legacy coordinates)."""
    n, h, w, c = x.shape
    oh, ow = int(size[0]), int(size[1])
    if out is None:
        out = torch.empty((n, oh, ow, c), dtype=x.dtype, device=x.device)
    xv, yv = nhwc(x), nhwc(out)
    check(lib().vm_resize_bilinear_tf1_nhwc(ctypes.byref(xv), ctypes.byref(yv), stream_handle()), "resize")
    return out


def convert(x, out, scale=None, shift=None, act="none"):
    """Copy x into out (dtype change, zero-filled extra channels, optional affine + activation)."""
    xv, yv = nhwc(x), nhwc(out)
    check(lib().vm_convert_nhwc(ctypes.byref(xv), ctypes.byref(yv), _ptr(_f32(scale)), _ptr(_f32(shift)),
                                _lib.ACT[act], stream_handle()), "convert")
    return out


_ws_cache = {}
_masked_streams = {}


_beside = {}


def _runs_beside(main, side, spin_us=1500):
    """True when a short kernel queued on ``side`` finishes while one queued before it on ``main`` still spins."""
    torch.cuda.synchronize(main.device)
    check(lib().vm_spin(spin_us, ctypes.c_void_p(main.cuda_stream)), "spin")
    e_main = torch.cuda.Event()
    e_main.record(main)
    check(lib().vm_spin(1, ctypes.c_void_p(side.cuda_stream)), "spin")
    e_side = torch.cuda.Event()
    e_side.record(side)
    beside = False
    while not e_main.query():
        if e_side.query():
            beside = True
            break
    torch.cuda.synchronize(main.device)
    return beside


def concurrent_streams(device, n, tries=16):
    """``n`` distinct pooled streams that each run beside the caller's current stream (as concurrent_stream; the
    candidates that share the caller's hardware queue are skipped), cached per (device, caller stream, n)."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    main = torch.cuda.current_stream(idx)
    key = (idx, main.cuda_stream, "n", n)
    got = _beside.get(key)
    if got is None:
        got, last = [], None
        for _ in range(tries):
            last = torch.cuda.Stream(device=torch.device("cuda", idx))
            if _runs_beside(main, last):
                got.append(last)
                if len(got) == n:
                    break
        while len(got) < n:  # (the probe kept failing: plain pool streams, slower at worst, never wrong)
            got.append(torch.cuda.Stream(device=torch.device("cuda", idx)))
        _beside[key] = got
    return list(got)


def concurrent_stream(device, tries=8):
    """A pooled torch stream that runs beside the caller's current stream of ``device``: a plain stream takes one of
    the process's hardware queues (GPU_MAX_HW_QUEUES) with no say in which, and on the caller's own queue a side
    stream's work is serialised behind the caller's (kernel traces).  Probed once per (device, current
    stream) with vm_spin; the chosen stream is cached and shared."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    main = torch.cuda.current_stream(idx)
    key = (idx, main.cuda_stream)
    s = _beside.get(key)
    if s is None:
        for _ in range(tries):
            s = torch.cuda.Stream(device=torch.device("cuda", idx))
            if _runs_beside(main, s):
                break
        _beside[key] = s  # (after `tries` misses: the last one; the step is then only slower, never wrong)
    return s


def side_stream(device, slot=0):
    """A CU-masked side stream of ``device`` (vm_stream_create_masked), one per ``slot``, created once per process and
    shared by the trainers that ask for that slot.  A plain torch stream takes one of the process's hardware queues
    without a say in which: a kernel trace caught a UNetImage trainer whose side stream sat on the caller's queue,
    serialising its filter gradients behind the data-gradient chain."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _masked_streams.get((idx, slot))
    if s is None:
        ptr = ctypes.c_void_p()
        with torch.cuda.device(idx):
            check(lib().vm_stream_create_masked(ctypes.byref(ptr)), "stream_create_masked")
        s = torch.cuda.ExternalStream(ptr.value, device=torch.device("cuda", idx))
        _masked_streams[(idx, slot)] = s
    return s


def _workspace(nbytes, device):
    key = (str(device), _lib.current_raw_stream(device.index if isinstance(device, torch.device) else None))
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def bn_stats(x, mean=None, var=None):
    """Batch mean / biased variance over N,H,W (tf.contrib batch_norm, is_training=True)."""
    c = x.shape[-1]
    mean = torch.empty(c, dtype=torch.float32, device=x.device) if mean is None else mean
    var = torch.empty(c, dtype=torch.float32, device=x.device) if var is None else var
    xv = nhwc(x)
    ws = _workspace(lib().vm_bn_workspace_bytes(ctypes.byref(xv)), x.device)
    check(lib().vm_bn_stats_nhwc(ctypes.byref(xv), _ptr(mean), _ptr(var), _ptr(ws), stream_handle()), "bn_stats")
    return mean, var


def bn_apply(x, mean, var, gamma, beta, eps=1e-3, act="none", out=None):
    out = x if out is None else out
    xv, yv = nhwc(x), nhwc(out)
    check(lib().vm_bn_apply_nhwc(ctypes.byref(xv), ctypes.byref(yv), _ptr(mean), _ptr(var), _ptr(gamma),
                                 _ptr(beta), float(eps), _lib.ACT[act], stream_handle()), "bn_apply")
    return out


def softmax_lastdim(x, out=None):
    out = torch.empty_like(x) if out is None else out
    xv, yv = nhwc(x), nhwc(out)
    check(lib().vm_softmax_lastdim_nhwc(ctypes.byref(xv), ctypes.byref(yv), stream_handle()), "softmax")
    return out



def composite_image(fg, bg, alpha, out_dtype=torch.float64, out=None):
    """vm_composite_image: reader.create_composite_image (reader.py:72-79) on the device.

    fg, bg: [..., cn] uint8 / float32 / float64 (same dtype); alpha: [...] float32 / float64.  Computed in
    float64 like numpy; out_dtype float64 (bit-identical to the reference) or float32.
    """
    _require_gpu(fg)
    if bg.shape != fg.shape or bg.dtype != fg.dtype or bg.device != fg.device:
        raise ValueError("composite_image: fg and bg must have the same shape, dtype and device")
    if fg.dim() < 1 or tuple(alpha.shape) != tuple(fg.shape[:-1]):
        raise ValueError("composite_image: alpha must be fg.shape[:-1], got %s vs %s" % (tuple(alpha.shape), tuple(fg.shape)))
    if fg.dtype not in (torch.uint8, torch.float32, torch.float64) or alpha.dtype not in (torch.float32, torch.float64):
        raise TypeError("composite_image: u8/f32/f64 images and f32/f64 alpha expected")
    if out_dtype not in (torch.float32, torch.float64):
        raise TypeError("composite_image: out_dtype must be float32 or float64")
    fg, bg, alpha = fg.contiguous(), bg.contiguous(), alpha.contiguous()
    if out is None:
        out = torch.empty(fg.shape, dtype=out_dtype, device=fg.device)
    elif out.shape != fg.shape or out.dtype != out_dtype or not out.is_contiguous():
        raise ValueError("composite_image: out must be a contiguous %s tensor of fg's shape" % out_dtype)
    cn = fg.shape[-1]
    check(lib().vm_composite_image(_ptr(fg), _ptr(bg), _AUG_DT[fg.dtype], _ptr(alpha), _AUG_DT[alpha.dtype],
                                   fg.numel() // max(cn, 1), cn, _ptr(out), _AUG_DT[out_dtype], stream_handle()),
          "composite_image")
    return out


# ---------------------------------------------------------------------------------------------- flow

def remap_f32(img, flow, mode="opencv", out=None):
    """Backward warp of single-channel f32 frames: img [n?,ih,iw], flow [n?,h,w,2] -> [n?,h,w]."""
    _require_gpu(img)
    _require_gpu(flow)
    batched = flow.dim() == 4
    f = flow if batched else flow[None]
    im = img if img.dim() == 3 else img[None]
    n, h, w, two = f.shape
    if two != 2 or im.shape[0] != n:
        raise ValueError("flow must be [h,w,2] (or [n,h,w,2]) matching img frames")
    im = im.contiguous().float()
    f = f.contiguous().float()
    if out is None:
        out = torch.empty((n, h, w), dtype=torch.float32, device=img.device)
    check(lib().vm_remap_bilinear_f32(_ptr(im), im.shape[1], im.shape[2], _ptr(f), h, w, n, _ptr(out),
                                      0 if mode == "opencv" else 1, stream_handle()), "remap_f32")
    return out if batched else out[0]


def remap_u8(img, flow):
    _require_gpu(img)
    _require_gpu(flow)
    img = img.contiguous()
    ih, iw = img.shape[:2]
    cn = 1 if img.dim() == 2 else img.shape[2]
    h, w = flow.shape[:2]
    out = torch.empty((h, w) + (() if img.dim() == 2 else (cn,)), dtype=torch.uint8, device=img.device)
    f = flow.contiguous().float()
    check(lib().vm_remap_bilinear_u8(_ptr(img), ih, iw, cn, _ptr(f), h, w, _ptr(out), stream_handle()), "remap_u8")
    return out


def fb_consistency(backward, forward, alpha, thresh=15.0, promote="numpy1"):
    """flow.correct_alpha on device; alpha (f32 [h,w], contiguous) is modified in place."""
    for t in (backward, forward, alpha):
        _require_gpu(t)
    h, w = backward.shape[:2]
    if alpha.dtype != torch.float32 or not alpha.is_contiguous() or tuple(alpha.shape) != (h, w):
        raise ValueError("alpha must be a contiguous f32 [h,w] device tensor")
    bw = backward.contiguous().float()
    fw = forward.contiguous().float()
    err = torch.zeros(1, dtype=torch.int32, device=alpha.device)
    check(lib().vm_fb_consistency(_ptr(bw), _ptr(fw), h, w, _ptr(alpha), float(thresh),
                                  0 if promote == "numpy1" else 1, _ptr(err), stream_handle()), "fb_consistency")
    if int(err.item()) != 0:
        raise IndexError("correct_alpha: a backward-flow target lies more than one frame outside the image "
                         "(the reference's numpy IndexError, flow.py:46)")
    return alpha


def matting_loss(pred, gt, raw_fg, in_bg, in_cmp):
    """train.py:42-47 loss on device -> tensor [loss, alpha_loss, compositional_loss]."""
    ts = [t.contiguous().float() for t in (pred, gt, raw_fg, in_bg, in_cmp)]
    for t in ts:
        _require_gpu(t)
    pixels = ts[0].numel()
    out = torch.empty(3, dtype=torch.float32, device=pred.device)
    ws = _workspace(lib().vm_loss_workspace_bytes(pixels), pred.device)
    check(lib().vm_matting_loss(*[_ptr(t) for t in ts], pixels, _ptr(out), _ptr(ws), stream_handle()),
          "matting_loss")
    return out


# ---------------------------------------------------------------- augmentation row (tps.py / augmentation.py)

_AUG_DT = {torch.uint8: _lib.VM_U8, torch.float32: _lib.VM_F32, torch.float64: _lib.VM_F64}


def _dtype_code(t, what):
    if t.dtype not in _AUG_DT:
        raise TypeError("%s: unsupported dtype %s (uint8, float32, float64)" % (what, t.dtype))
    return _AUG_DT[t.dtype]


def tps_grid(points, coeffs, nx, ny, x_lo, x_step, y_lo, y_step, out=None):
    """vm_tps_grid: the TPS map evaluated on an nx x ny np.mgrid lattice -> f64 [2, nx, ny] on the device."""
    _require_gpu(points)
    _require_gpu(coeffs)
    p = points.contiguous().double()
    c = coeffs.contiguous().double()
    if p.dim() != 2 or p.shape[1] != 2 or c.shape != (p.shape[0] + 3, 2):
        raise ValueError("tps_grid: points [n,2] and coeffs [n+3,2], got %s %s" % (tuple(p.shape), tuple(c.shape)))
    if out is None:
        out = torch.empty((2, nx, ny), dtype=torch.float64, device=p.device)
    check(lib().vm_tps_grid(_ptr(p), _ptr(c), p.shape[0], nx, ny, float(x_lo), float(x_step), float(y_lo),
                            float(y_step), _ptr(out), stream_handle()), "tps_grid")
    return out


def tps_sample(grid, img, order=1, upsample=None, out=None):
    """vm_tps_sample: map_coordinates of img [ih, iw, cn] (u8/f32/f64) through the grid (or its upsampling:
    upsample = (x_steps, x_span, y_steps, y_span)) -> [oh, ow, cn] of img's dtype."""
    _require_gpu(grid)
    _require_gpu(img)
    img = img.contiguous()
    if img.dim() == 2:
        img = img[:, :, None]
    ih, iw, cn = img.shape
    nx, ny = grid.shape[1:]
    m = _lib.VmTpsMap()
    m.grid = _ptr(grid)
    m.nx, m.ny = nx, ny
    if upsample is None:
        m.upsample = 0
        oh, ow = nx, ny
    else:
        xs, xspan, ys, yspan = upsample
        m.upsample, m.x_steps, m.x_span, m.y_steps, m.y_span = 1, float(xs), int(xspan), float(ys), int(yspan)
        oh, ow = int(xspan) + 1, int(yspan) + 1
    if out is None:
        out = torch.empty((oh, ow, cn), dtype=img.dtype, device=img.device)
    check(lib().vm_tps_sample(ctypes.byref(m), _ptr(img), ih, iw, cn, _dtype_code(img, "tps_sample"), int(order),
                              _ptr(out), stream_handle()), "tps_sample")
    return out


def warp_affine(src, M, dsize, out=None):
    """vm_warp_affine: cv2.warpAffine(src, M, dsize=(w, h)), INTER_LINEAR, BORDER_CONSTANT 0."""
    _require_gpu(src)
    src = src.contiguous()
    two_d = src.dim() == 2
    ih, iw = src.shape[:2]
    cn = 1 if two_d else src.shape[2]
    w, h = int(dsize[0]), int(dsize[1])
    m = (ctypes.c_double * 6)(*[float(v) for v in np.asarray(M, np.float64).reshape(6)])
    if out is None:
        out = torch.empty((h, w) if two_d else (h, w, cn), dtype=src.dtype, device=src.device)
    check(lib().vm_warp_affine(_ptr(src), ih, iw, cn, _dtype_code(src, "warp_affine"), m, _ptr(out), h, w,
                               stream_handle()), "warp_affine")
    return out


def warp_image(src, tu, tv, M, dsize, lut=None, out=None):
    """vm_warp_image: augmentation.warp_image's translate + warpAffine pair (augmentation.py:59-63) in one pass,
    optionally followed by change_illumination with the S/V map ``lut`` (u8 BGR)."""
    _require_gpu(src)
    src = src.contiguous()
    two_d = src.dim() == 2
    ih, iw = src.shape[:2]
    cn = 1 if two_d else src.shape[2]
    w, h = int(dsize[0]), int(dsize[1])
    m = (ctypes.c_double * 6)(*[float(v) for v in np.asarray(M, np.float64).reshape(6)])
    lp = None
    if lut is not None:
        lut = np.ascontiguousarray(lut, np.uint8)
        if lut.shape != (256,):
            raise ValueError("warp_image: lut must have 256 entries")
        lp = lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    if out is None:
        out = torch.empty((h, w) if two_d else (h, w, cn), dtype=src.dtype, device=src.device)
    check(lib().vm_warp_image(_ptr(src), ih, iw, cn, _dtype_code(src, "warp_image"), int(tu), int(tv), m, lp,
                              _ptr(out), h, w, stream_handle()), "warp_image")
    return out


def change_illumination(bgr, lut, out=None):
    """vm_change_illumination_u8: BGR u8 -> HSV -> (h, lut[s], lut[v]) -> BGR u8."""
    _require_gpu(bgr)
    if bgr.dtype != torch.uint8 or bgr.shape[-1] != 3:
        raise TypeError("change_illumination: uint8 [..., 3] expected")
    bgr = bgr.contiguous()
    lut = np.ascontiguousarray(lut, np.uint8)
    if lut.shape != (256,):
        raise ValueError("change_illumination: lut must have 256 entries")
    if out is None:
        out = torch.empty_like(bgr)
    check(lib().vm_change_illumination_u8(_ptr(bgr), bgr.numel() // 3,
                                          lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _ptr(out),
                                          stream_handle()), "change_illumination")
    return out


def bgra(fg, alpha, out=None):
    """vm_bgra_u8: concat(fg u8 [h, w, 3], uint8(255. * alpha [h, w] f64 / f32)) -> u8 [h, w, 4]."""
    _require_gpu(fg)
    _require_gpu(alpha)
    fg, alpha = fg.contiguous(), alpha.contiguous()
    h, w = fg.shape[:2]
    if fg.dtype != torch.uint8 or tuple(fg.shape) != (h, w, 3) or alpha.numel() != h * w:
        raise ValueError("bgra: fg u8 [h, w, 3] and alpha [h, w]")
    if out is None:
        out = torch.empty((h, w, 4), dtype=torch.uint8, device=fg.device)
    check(lib().vm_bgra_u8(_ptr(fg), _ptr(alpha), _dtype_code(alpha, "bgra"), h * w, _ptr(out), stream_handle()),
          "bgra")
    return out


def nonzero_stats(alpha, out=None):
    """vm_nonzero_stats: (count, row-index sum, column-index sum) of alpha != 0, int64[3] on the device."""
    _require_gpu(alpha)
    alpha = alpha.contiguous()
    if alpha.dim() != 2:
        raise ValueError("nonzero_stats: alpha must be [h, w]")
    if out is None:
        out = torch.empty(3, dtype=torch.int64, device=alpha.device)
    check(lib().vm_nonzero_stats(_ptr(alpha), alpha.shape[0], alpha.shape[1], _dtype_code(alpha, "nonzero_stats"),
                                 _ptr(out), stream_handle()), "nonzero_stats")
    return out


def trimap_from_matte(matte, dilate=1, crop=3, out=None):
    """vm_trimap_from_matte: data.trimap_from_matte on a float64 [h, w] device matte -> uint8 [h, w]."""
    _require_gpu(matte)
    if matte.dtype != torch.float64 or matte.dim() != 2:
        raise AssertionError("trimap_from_matte: float64 [h, w] matte expected (data.py:42)")
    matte = matte.contiguous()
    if out is None:
        out = torch.empty(matte.shape, dtype=torch.uint8, device=matte.device)
    check(lib().vm_trimap_from_matte(_ptr(matte), matte.shape[0], matte.shape[1], int(dilate), int(crop), _ptr(out),
                                     stream_handle()), "trimap_from_matte")
    return out


# ---------------------------------------------------------------- training step (train.py:288-343, config 5)

def matting_loss_backward(pred, gt, raw_fg, in_bg, in_cmp, out=None):
    """dL/dlogits of train.py:294-298's loss for pred = sigmoid(logits) (all contiguous f32 device tensors)."""
    ts = [_f32(t) for t in (pred, gt, raw_fg, in_bg, in_cmp)]
    pixels = ts[0].numel()
    if ts[1].numel() != pixels or any(t.numel() != 3 * pixels for t in ts[2:]):
        raise ValueError("matting_loss_backward: pred/gt [P], raw_fg/bg/cmp [P,3]")
    out = torch.empty_like(ts[0]) if out is None else _f32(out)
    check(lib().vm_matting_loss_backward(*[_ptr(t) for t in ts], pixels, _ptr(out), stream_handle()),
          "matting_loss_backward")
    return out


def bn_backward(x, dy, y, mean, var, gamma, eps=1e-3, dx=None, dgamma=None, dbeta=None, dx2=None, dbias=None):
    """Gradient of tf.contrib batch_norm(is_training=True) (+ the relu after it when ``y`` is given).
    x None: only dbeta = channel sum of dy (a bias gradient).  dx2: optional second copy of dx (e.g. bf16).
    dbias: the gradient of a conv bias added before the BN (= channel sum of dx) from the same reduction."""
    c = dy.shape[-1]
    views = [None if t is None else nhwc(t) for t in (x, dy, y, dx, dx2)]
    ref = lambda v: None if v is None else ctypes.byref(v)  # noqa: E731
    ws = _workspace(lib().vm_bn_backward_workspace_bytes(c), dy.device)
    check(lib().vm_bn_backward_ex_nhwc(ref(views[0]), ref(views[1]), ref(views[2]), _ptr(mean), _ptr(var),
                                       _ptr(gamma), float(eps), ref(views[3]), ref(views[4]), _ptr(dgamma),
                                       _ptr(dbeta), _ptr(dbias), _ptr(ws), stream_handle()), "bn_backward")
    return dx


def bn_backward_apply(x, dy, y, mean, var, gamma, sum_g, sum_gx, count, dx, eps=1e-3, dx2=None):
    """The input-gradient pass of bn_backward with given channel sums over ``count`` pixels (SyncBN: the sums
    all-reduced over the replicas, count = their pixels)."""
    views = [None if t is None else nhwc(t) for t in (x, dy, y, dx, dx2)]
    ref = lambda v: None if v is None else ctypes.byref(v)  # noqa: E731
    check(lib().vm_bn_backward_apply_nhwc(ref(views[0]), ref(views[1]), ref(views[2]), _ptr(mean), _ptr(var),
                                          _ptr(gamma), float(eps), _ptr(_f32(sum_g)), _ptr(_f32(sum_gx)), int(count),
                                          ref(views[3]), ref(views[4]), stream_handle()), "bn_backward_apply")
    return dx


def relu_backward(dy, y, dx, dx2=None, dx_lo=None):
    """dx = dy * (y > 0) (+ a second copy dx2, e.g. bf16).  ``dx_lo``: its channels k = dx_lo.shape[-1] take the
    first k channels of the gradient and dx / dx2 the rest (one pass over a decoder level's concat)."""
    dv, yv, xv = nhwc(dy), nhwc(y), nhwc(dx)
    x2 = ctypes.byref(nhwc(dx2)) if dx2 is not None else None
    if dx_lo is None:
        check(lib().vm_relu_backward_ex_nhwc(ctypes.byref(dv), ctypes.byref(yv), ctypes.byref(xv), x2,
                                             stream_handle()), "relu_backward")
        return dx
    lv = nhwc(dx_lo)
    check(lib().vm_relu_backward_split_nhwc(ctypes.byref(dv), ctypes.byref(yv), dx_lo.shape[-1], ctypes.byref(lv),
                                            ctypes.byref(xv), x2, stream_handle()), "relu_backward")
    return dx


def maxpool_backward(x, dy, dx, add=None):
    """Adjoint of maxpool2x2 (tf.nn.max_pool 2x2/2 SAME): dx = add + dy routed to each window's first maximum of x
    (TF MaxPoolGrad's tie rule).  ``add`` may be dx itself."""
    xv, dv, ov = nhwc(x), nhwc(dy), nhwc(dx)
    av = ctypes.byref(nhwc(add)) if add is not None else None
    check(lib().vm_maxpool2x2_backward_nhwc(ctypes.byref(xv), ctypes.byref(dv), av, ctypes.byref(ov),
                                            stream_handle()), "maxpool_backward")
    return dx


def relu_backward_bias(dy, y, dz, dbias, add=None):
    """vm_relu_backward_bias_nhwc: dz = (y > 0) * g and dbias = channel sums of dz in one pass; g = dy (+ add), or —
    when dy has the 2x2 SAME pool's shape — add + the max-pool adjoint of dy (TF MaxPoolGrad's first maximum)."""
    _f32(dbias)
    views = [nhwc(dy), nhwc(y), None if add is None else nhwc(add), nhwc(dz)]
    ref = lambda v: None if v is None else ctypes.byref(v)  # noqa: E731
    ws = _workspace(lib().vm_relu_backward_bias_workspace_bytes(y.shape[-1]), y.device)
    check(lib().vm_relu_backward_bias_nhwc(ref(views[0]), ref(views[1]), ref(views[2]), ref(views[3]), _ptr(dbias),
                                           _ptr(ws), stream_handle()), "relu_backward_bias")
    return dz


def resize_backward(dy, dx):
    """Adjoint of resize_bilinear: dy [n,oh,ow,c] -> dx contiguous f32 (or bf16, c % 4 == 0) [n,ih,iw,c]
    (overwritten)."""
    if dx.shape[0] != dy.shape[0] or dx.shape[3] != dy.shape[3]:
        raise ValueError("resize_backward: batch/channel mismatch")
    dv = nhwc(dy)
    if dx.dtype == torch.bfloat16:
        xv = nhwc(dx)
        check(lib().vm_resize_bilinear_tf1_backward_nhwc(ctypes.byref(dv), ctypes.byref(xv), stream_handle()),
              "resize_backward")
        return dx
    _f32(dx)
    check(lib().vm_resize_bilinear_tf1_backward(ctypes.byref(dv), _ptr(dx), dx.shape[1], dx.shape[2],
                                                stream_handle()), "resize_backward")
    return dx


def conv_wgrad(x, dy, dw, mfma=False, sources=None):
    """dw[3,3,cin,cout] += 3x3 SAME conv weight gradient of input view x and output-gradient view dy (f32; bf16 too
    for the wide MFMA kernel, cout > 48).

    ``mfma``: bf16 x only — the MFMA kernel with dy rounded to bf16 (the bf16 training path); else the exact-f32
    FMA kernel.  ``sources`` = (number of sources, element stride between sources): x is the [n,h,w,c] view of
    source 0 and the conv input is the channel concat of the sources (tower-major features, MFMA kernel only)."""
    _f32(dw)
    if isinstance(x, SourceConcat):
        x, sources = x.src0, (x.nsrc, x.stride)
    n, h, w, cin = x.shape
    cout = dy.shape[-1]
    src_c = cin
    if sources is not None:
        cin = src_c * int(sources[0])
    if tuple(dy.shape[:3]) != (n, h, w) or dw.numel() != 9 * cin * cout:
        raise ValueError("conv_wgrad: x %s, dy %s, dw %s" % (tuple(x.shape), tuple(dy.shape), tuple(dw.shape)))
    dv = nhwc(dy)
    if mfma or sources is not None or cout > 48:  # (cout > 48: the wide kernels, UNetImage training)
        xv = nhwc(x)
        xv.c = cin
        src_c, stride = (src_c, int(sources[1])) if sources is not None else (0, 0)
        mode = 1 if mfma else 0
        ws = _workspace(lib().vm_conv3x3_wgrad_ex_workspace_bytes(n, h, w, cin, cout, mode), x.device)
        check(lib().vm_conv3x3_wgrad_ex_nhwc(ctypes.byref(xv), src_c, stride, ctypes.byref(dv), _ptr(dw), _ptr(ws),
                                             mode, stream_handle()), "conv_wgrad_ex")
        return dw
    xv = nhwc(x)
    ws = _workspace(lib().vm_conv3x3_wgrad_workspace_bytes(n, h, w, cin, cout), x.device)
    check(lib().vm_conv3x3_wgrad_nhwc(ctypes.byref(xv), ctypes.byref(dv), _ptr(dw), _ptr(ws), stream_handle()),
          "conv_wgrad")
    return dw


def flip_weights(w_hwio, out):
    cin, cout = int(w_hwio.shape[2]), int(w_hwio.shape[3])
    check(lib().vm_conv3x3_flip_weights(_ptr(_f32(w_hwio)), cin, cout, _ptr(_f32(out)), stream_handle()),
          "flip_weights")
    return out


def adam_tf(var, m, v, grad, lr_t, beta1, beta2, eps, grad_scale=1.0):
    for t in (var, m, v, grad):
        _f32(t)
    check(lib().vm_adam_tf(_ptr(var), _ptr(m), _ptr(v), _ptr(grad), var.numel(), float(lr_t), float(beta1),
                           float(beta2), float(eps), float(grad_scale), stream_handle()), "adam")
    return var
