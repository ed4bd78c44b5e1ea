"""ctypes binding of libmsl_hip.so (the C-ABI declared in include/msl_hip.h).

This is the only place the product path reaches native code.  There is no
fallback: if the library is missing or no GPU is visible, every compute call
raises.  `import torch` happens before the library is loaded so that its
libamdhip64.so.7 dependency resolves to the HIP runtime torch already mapped
(one runtime per process, so torch's hipStream_t handles are valid here).
"""
import ctypes
import os

import torch

# MSL_LIB_PATH: another build of the same library (same-box A/B of kernel changes, scripts/bench_ops.py)
LIB_PATH = os.environ.get("MSL_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                          "libmsl_hip.so")

c_int, c_ll, c_sz, c_f, c_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_float, ctypes.c_void_p

# name -> (restype, argtypes); must match include/msl_hip.h exactly.
SIGNATURES = {
    "msl_abi_version": (c_int, []),
    "msl_status_string": (ctypes.c_char_p, [c_int]),
    "msl_dconv_packed_elems": (c_ll, [c_int, c_int, c_int, c_int]),
    "msl_forms_default": (c_int, [c_p]),
    "msl_forms_check": (c_int, [c_p]),
    "msl_dconv_pack": (c_int, [c_p, c_ll, c_int, c_int, c_int, c_int, c_p, c_p, c_p]),
    "msl_conv_pack_blocks": (c_ll, [c_int] * 5),
    "msl_conv_pack_many": (c_int, [c_p, c_p, c_int, c_int, c_ll, c_p, c_p]),
    "msl_dconv_fwd_workspace": (c_sz, [c_int] * 6),
    "msl_dconv_fwd": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p]),
    "msl_dconv_dgrad_workspace": (c_sz, [c_int] * 6),
    "msl_dconv_dgrad": (c_int, [c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p]),
    "msl_dconv_wgrad_workspace": (c_sz, [c_int] * 6),
    "msl_dconv_wgrad": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 9 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_packed_elems": (c_ll, [c_int] * 3),
    "msl_pconv_pack": (c_int, [c_p, c_int, c_int, c_int, c_p, c_p, c_p]),
    "msl_pconv_fwd_workspace": (c_sz, [c_int] * 3),
    "msl_pconv_fwd": (c_int, [c_p, c_p, c_p] + [c_int] * 3 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_dgrad_workspace": (c_sz, [c_int] * 3),
    "msl_pconv_dgrad": (c_int, [c_p, c_p, c_p] + [c_int] * 3 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_dgrad_acc": (c_int, [c_p, c_p, c_p] + [c_int] * 4 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_wgrad_workspace": (c_sz, [c_int] * 3),
    "msl_pconv_wgrad": (c_int, [c_p, c_p, c_p] + [c_int] * 4 + [c_p, c_p, c_sz, c_p]),
    "msl_absmax_partials": (c_int, [c_p, c_int, c_int, c_p, c_p]),
    "msl_dconv_fwd_sc": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_dconv_dgrad_sc": (c_int, [c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_dconv_wgrad_sc": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 9 + [c_p, c_p, c_sz, c_p, c_p, c_int, c_p, c_int]),
    "msl_pconv_fwd_sc": (c_int, [c_p, c_p, c_p] + [c_int] * 3 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_pconv_dgrad_acc_sc": (c_int, [c_p, c_p, c_p] + [c_int] * 4 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_pconv_wgrad_sc": (c_int, [c_p, c_p, c_p] + [c_int] * 4 + [c_p, c_p, c_sz, c_p, c_p, c_int, c_p, c_int]),
    "msl_dconv_fwd_f16": (c_int, [c_p] * 4 + [c_int] * 8 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_dconv_dgrad_f16": (c_int, [c_p] * 3 + [c_int] * 8 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_dconv_wgrad_f16": (c_int, [c_p] * 4 + [c_int] * 9 + [c_p, c_p, c_sz, c_p, c_p, c_int, c_p, c_int]),
    "msl_pconv_fwd_f16": (c_int, [c_p] * 3 + [c_int] * 3 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_pconv_dgrad_f16": (c_int, [c_p] * 3 + [c_int] * 4 + [c_p, c_p, c_sz, c_p, c_p, c_int]),
    "msl_pconv_wgrad_f16": (c_int, [c_p] * 3 + [c_int] * 4 + [c_p, c_p, c_sz, c_p, c_p, c_int, c_p, c_int]),
    "msl_conv_wgrad_split": (c_int, [c_int] * 7),
    "msl_dconv_fwd_bf16": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p]),
    "msl_dconv_dgrad_bf16": (c_int, [c_p, c_p, c_p] + [c_int] * 8 + [c_p, c_p, c_sz, c_p]),
    "msl_dconv_wgrad_bf16": (c_int, [c_p, c_p, c_p, c_p] + [c_int] * 9 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_fwd_bf16": (c_int, [c_p, c_p, c_p] + [c_int] * 3 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_dgrad_bf16": (c_int, [c_p, c_p, c_p] + [c_int] * 3 + [c_p, c_p, c_sz, c_p]),
    "msl_pconv_wgrad_bf16": (c_int, [c_p, c_p, c_p] + [c_int] * 4 + [c_p, c_p, c_sz, c_p]),
    "msl_upsample_fwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_p]),
    "msl_upsample_bwd_workspace": (c_sz, [c_int] * 5),
    "msl_upsample_bwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_p, c_sz, c_p]),
    "msl_loss_workspace": (c_sz, [c_int] * 5),
    "msl_loss_stats_elems": (c_int, []),
    "msl_ce_up_fwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_p, c_p, c_p, c_sz, c_p]),
    "msl_ce_up_bwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_maxsquare_up_fwd": (c_int, [c_p] + [c_int] * 5 + [c_p, c_p, c_p, c_sz, c_p]),
    "msl_maxsquare_up_bwd": (c_int, [c_p] + [c_int] * 5 + [c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_iw_maxsquare_up_fwd": (c_int, [c_p] + [c_int] * 5 + [c_f, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_iw_maxsquare_up_bwd": (c_int, [c_p] + [c_int] * 5 + [c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_multi_ce_up_fwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_f, c_p, c_p, c_p, c_sz, c_p]),
    "msl_multi_ce_up_bwd": (c_int, [c_p, c_p] + [c_int] * 5 + [c_f, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_loss_labels_up": (c_int, [c_p, c_p] + [c_int] * 5 + [c_f, c_p, c_p, c_p]),
    "msl_maxsquare_prob_fwd": (c_int, [c_p, c_int, c_int, c_p, c_p, c_sz, c_p]),
    "msl_maxsquare_prob_bwd": (c_int, [c_p, c_int, c_int, c_p, c_p, c_p]),
    "msl_iw_maxsquare_prob_fwd": (c_int, [c_p, c_p, c_int, c_int, c_f, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "msl_iw_maxsquare_prob_bwd": (c_int, [c_p, c_int, c_int, c_p, c_p, c_p, c_p]),
    "msl_confusion_accumulate": (c_int, [c_p, c_p, c_int, ctypes.c_longlong, c_p, c_p, c_p]),
    "msl_bn_uses_fused": (c_int, [c_int, c_int, c_int, c_p]),
    "msl_bn_workspace": (c_sz, [c_int] * 3),
    "msl_bn_fwd": (c_int, [c_p] * 10 + [c_int] * 5 + [c_f, c_f, c_int, c_p, c_p, c_sz, c_p]),
    "msl_bn_bwd": (c_int, [c_p] * 10 + [c_int] * 6 + [c_p, c_p, c_sz, c_p]),
    "msl_bn_fwd_am": (c_int, [c_p] * 10 + [c_int] * 5 + [c_f, c_f, c_int, c_p, c_p, c_sz, c_p, c_p]),
    "msl_bn_bwd_am": (c_int, [c_p] * 10 + [c_int] * 6 + [c_p, c_p, c_sz, c_p, c_p]),
    "msl_bn_bwd_am_beta": (c_int, [c_p] * 11 + [c_int] * 6 + [c_p, c_p, c_sz, c_p, c_p]),
    "msl_bn_relu_mask_bytes": (c_sz, [c_int] * 3),
    "msl_bn_fwd_mask": (c_int, [c_p] * 10 + [c_int] * 5 + [c_f, c_f, c_int, c_p, c_p, c_sz, c_p, c_p, c_p]),
    "msl_bn_bwd_mask": (c_int, [c_p] * 11 + [c_int] * 6 + [c_p, c_p, c_sz, c_p, c_p]),
    "msl_image_transform": (c_int, [c_p, c_int, c_int, c_int, c_f, c_f, c_f, c_p, c_p]),
    "msl_label_transform": (c_int, [c_p, c_int, c_int, c_int, c_p, c_p, c_p]),
    "msl_im2col": (c_int, [c_p] + [c_int] * 11 + [c_p, c_p]),
    "msl_col2im": (c_int, [c_p] + [c_int] * 11 + [c_p, c_p]),
    "msl_maxpool_fwd": (c_int, [c_p] + [c_int] * 8 + [c_p, c_p, c_p]),
    "msl_maxpool_bwd": (c_int, [c_p, c_p] + [c_int] * 8 + [c_p, c_p]),
    "msl_subsample": (c_int, [c_p] + [c_int] * 6 + [c_p, c_p]),
    "msl_subsample_bwd": (c_int, [c_p] + [c_int] * 6 + [c_p, c_p]),
    "msl_aspp_weight_layout": (c_int, [c_p, c_ll, c_int, c_int, c_int, c_p, c_p]),
    "msl_aspp_weight_grad": (c_int, [c_p, c_int, c_int, c_int, c_p, c_p]),
    "msl_aspp_shift_add": (c_int, [c_p, c_p, c_p] + [c_int] * 7 + [c_p]),
    "msl_aspp_shift_gather": (c_int, [c_p, c_p, c_p] + [c_int] * 7 + [c_p]),
    "msl_sgd_block_elems": (c_int, []),
    "msl_sgd_plan": (c_ll, [c_p, c_int, c_p, c_p, c_ll]),
    "msl_sgd_step": (c_int, [c_p, c_p, c_p, c_ll, c_f, c_f, c_f, c_f, c_f, c_p]),
    "msl_sgd_step_lr_dev": (c_int, [c_p, c_p, c_p, c_ll, c_p, c_f, c_f, c_f, c_p]),
    "msl_launch_guard_probe": (c_int, [c_int, c_p, c_p]),
    "msl_pconv_dgrad_resmask_sc": (c_int, [c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_int, c_p, c_p, c_sz, c_p, c_p,
                                           c_int]),
    "msl_pconv_dgrad_resmask_f16": (c_int, [c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_int, c_p, c_p, c_sz, c_p,
                                            c_p, c_int]),
}

ABI_VERSION = 3
# r06 entry points an older build (MSL_LIB_PATH, a same-box A/B) may lack: the diagnostics probe and the masked
# residual dgrad (ops.py falls back to the materialised residual gradient without it)
_DIAGNOSTIC = {"msl_launch_guard_probe", "msl_pconv_dgrad_resmask_sc", "msl_pconv_dgrad_resmask_f16"}
_lib = None


class MSLError(RuntimeError):
    pass


_gpu_seen = False


def load(require_gpu=True):
    """Load libmsl_hip.so and declare every C-ABI symbol.  Raises if absent."""
    global _lib, _gpu_seen
    if require_gpu and not _gpu_seen:
        if not torch.cuda.is_available():
            raise MSLError("maxsquareloss_amd: no GPU visible; the HIP path has no CPU fallback")
        _gpu_seen = True  # a visible GPU stays visible: skip the per-op query
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MSLError(f"maxsquareloss_amd: {LIB_PATH} is missing; run __graft_entry__.build() "
                       "(make -C maxsquareloss_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if name in _DIAGNOSTIC and not hasattr(lib, name):
            continue  # an older build (MSL_LIB_PATH, a same-box A/B) without the diagnostics entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.msl_abi_version() != ABI_VERSION:
        raise MSLError("libmsl_hip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def check(status, what):
    if status != 0:
        msg = load(require_gpu=False).msl_status_string(status).decode()
        raise MSLError(f"{what} failed: {msg} (status {status})")


def stream_ptr():
    """torch's current HIP stream on the current device, as the raw hipStream_t every entry point
    takes (the direct accessor: torch.cuda.current_stream() costs ~8 us of Python per op)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def ptr(t):
    return None if t is None else t.data_ptr()


class Forms(ctypes.Structure):
    """msl_forms (include/msl_hip.h): the kernel forms every conv / pack / BN call takes (ABI 3)."""
    _fields_ = [("f32_form", c_int), ("sk_hybrid", c_int), ("pack_form", c_int), ("bn_fused", c_int)]


FORMS = Forms(5, 1, 1, 1)  # the forms this process passes: the library's defaults until set_form


def forms():
    """The const msl_forms* of every conv / pack / BN call: FORMS, read by the library on the host when
    the call launches (a captured graph keeps the forms of its capture)."""
    return ctypes.addressof(FORMS)


def snapshot_forms():
    """A copy of FORMS: an autograd function keeps the forms of its forward and passes them to
    its backward's calls, so a form switched between the two (the tests toggle them) cannot hand a
    backward kernel a state its forward did not leave (the fused BN's mask bits, a pack's form)."""
    return Forms(*(getattr(FORMS, f) for f, _ in Forms._fields_))


def set_form(name, value):
    """Set one field of FORMS (checked by msl_forms_check); returns the previous value."""
    trial = Forms(*(getattr(FORMS, f) for f, _ in Forms._fields_))
    setattr(trial, name, int(value))
    check(load(require_gpu=False).msl_forms_check(ctypes.addressof(trial)), f"msl_forms {name}={value}")
    prev = getattr(FORMS, name)
    setattr(FORMS, name, int(value))
    return prev


def workspace(nbytes, device):
    """Scratch from the caching allocator (stream-ordered reuse, no sync)."""
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
