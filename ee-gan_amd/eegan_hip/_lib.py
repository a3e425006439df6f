"""ctypes binding of libeegan_hip.so (the C ABI declared in include/eegan_hip.h).

The product path has no fallback: if the HIP library is missing or fails to
load, importing this module raises.  Every call checks the returned status
and raises RuntimeError with eegan_last_error()'s text.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('EEGAN_HIP_LIB', os.path.join(_HERE, 'libeegan_hip.so'))

ACT_NONE, ACT_RELU, ACT_LRELU, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3, 4
ACT_CODES = {None: 0, 'none': 0, 'relu': 1, 'lrelu': 2, 'tanh': 3, 'sigmoid': 4}


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int) for n in ['N', 'H', 'W', 'C', 'ldx', 'K', 'R', 'S', 'stride', 'pad_h', 'pad_w',
                                       'up2', 'Ho', 'Wo', 'ldy']] + [('splitk_ctr', C.c_void_p),
                                                                     ('splitk_ctr_n', C.c_int),
                                                                     ('plan', C.c_int)]


class BnModDesc(C.Structure):
    _fields_ = [('x', C.c_void_p), ('N', C.c_int), ('H', C.c_int), ('W', C.c_int), ('C', C.c_int),
                ('ldx', C.c_int), ('up2', C.c_int), ('stats', C.c_void_p), ('mode', C.c_int),
                ('w', C.c_void_p), ('b', C.c_void_p), ('gam', C.c_void_p), ('bet', C.c_void_p),
                ('mask', C.c_void_p), ('act', C.c_int), ('slope', C.c_float)]


class GemmDesc(C.Structure):
    _fields_ = [('A', C.c_void_p), ('B', C.c_void_p), ('C', C.c_void_p), ('bias', C.c_void_p),
                ('gate', C.c_void_p)] + [(n, C.c_long) for n in ['sai', 'sak', 'sbk', 'sbj', 'ldc', 'ldg']] + \
               [(n, C.c_int) for n in ['M', 'N', 'K', 'act', 'gate_act']] + [('alpha', C.c_float), ('beta', C.c_float)]


class ImgJob(C.Structure):
    _fields_ = [('src_off', C.c_long)] + [(n, C.c_int) for n in ['src_stride', 'row0', 'nrows', 'flip', 'hcoef_off',
                                                                  'hbound_off', 'hksize', 'vcoef_off', 'vbound_off',
                                                                  'vksize']]


class ScaleTable(C.Structure):
    _fields_ = [('size', C.c_int), ('ksize', C.c_int), ('hcoef', C.c_void_p), ('hbounds', C.c_void_p),
                ('vcoef', C.c_void_p), ('vbounds', C.c_void_p)]


P, I, L, F, D = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_double
CD, BD = C.POINTER(ConvDesc), C.POINTER(BnModDesc)

# name: (argtypes, restype); the trailing P of every compute entry is the hipStream_t
_SIGS = {
    'eegan_last_error': ([], C.c_char_p),
    'eegan_abi_version': ([], I),
    'eegan_event_create': ([P], I),
    'eegan_event_destroy': ([P], I),
    'eegan_stream_create': ([P, I], I),
    'eegan_stream_destroy': ([P], I),
    'eegan_event_record': ([P, P], I),
    'eegan_event_elapsed': ([P, P, P], I),
    'eegan_timing_arm': ([P, P, P, P], I),
    'eegan_timing_disarm': ([P], I),
    'eegan_conv_packed_elems': ([I, I, I, I, I], L),
    'eegan_conv_pack_weights': ([P, P, I, I, I, I, I, P, P], I),
    'eegan_conv_pack_multi_blocks': ([I, I, I, I, I], L),
    'eegan_conv_pack_weights_multi': ([P, I, L, P], I),
    'eegan_conv_fwd_workspace': ([CD], L),
    'eegan_conv_bwd_data_workspace': ([CD], L),
    'eegan_conv_fwd': ([CD, P, P, P, I, F, P, I, P, P, I, P, P], I),
    'eegan_conv_bwd_data': ([CD, P, P, P, I, I, P, P], I),
    'eegan_conv_bwd_data_gated': ([CD, P, P, P, I, I, P, I, I, F, P, P], I),
    'eegan_conv_bwd_data_ex': ([CD, P, P, P, I, I, P, I, I, F, P, I, I, F, P, P], I),
    'eegan_conv_wgrad_workspace': ([CD], L),
    'eegan_conv_bwd_weight': ([CD, P, P, P, P, I, P], I),
    'eegan_bn_stats_workspace': ([L, I], L),
    'eegan_bn_stats': ([P, L, I, I, P, P, P], I),
    'eegan_bn_finalize': ([P, I, D, D, F, F, I, P, P, P, P], I),
    'eegan_bnmod_fwd': ([BD, P, I, P], I),
    'eegan_bnmod_fwd_fin': ([BD, P, D, D, F, F, I, P, P, P, I, P], I),
    'eegan_bnmod_bwd_workspace': ([BD], L),
    'eegan_bnmod_bwd': ([BD, P, I, P, P, P, P, P, P], I),
    'eegan_bnmod_bwd_dx': ([BD, P, I, P, D, P, I, P], I),
    'eegan_act_bwd': ([P, I, P, I, L, I, I, F, P, I, P], I),
    'eegan_scale_add': ([P, I, P, I, P, F, L, I, P, I, P], I),
    'eegan_cat_channels': ([P, P, P, I, L, P, I, P], I),
    'eegan_scale_dot': ([P, I, P, I, P, F, L, I, P, I, P, P, I, I, F, P], I),
    'eegan_scale_dot_res': ([P, I, P, I, P, F, L, I, P, I, P, I, P, P, I, P], I),
    'eegan_scale_gate': ([P, I, P, I, I, F, P, F, L, I, P, I, P, I, P, I, P, P, I, P], I),
    'eegan_dot_workspace': ([], L),
    'eegan_dot': ([P, I, P, I, L, I, F, P, P, I, P], I),
    'eegan_chansum_workspace': ([L, I], L),
    'eegan_chansum': ([P, I, L, I, P, P, I, P], I),
    'eegan_avgpool2': ([P, I, I, I, I, I, P, I, P], I),
    'eegan_upsample2': ([P, I, I, I, I, I, F, P, I, P], I),
    'eegan_sumpool2': ([P, I, I, I, I, I, P, I, P], I),
    'eegan_cat_tile': ([P, I, P, I, I, I, I, P, I, P], I),
    'eegan_cat_tile_bwd': ([P, I, I, I, I, I, P, I, P, P], I),
    'eegan_bilinear': ([P, I, I, I, I, I, I, I, I, I, I, P, I, I, P], I),
    'eegan_bilinear_bwd': ([P, I, P, I, I, I, I, I, I, I, I, I, I, P, P], I),
    'eegan_convert': ([P, L, I, P, I, I, P], I),
    'eegan_nchw_to_nhwc': ([P, I, I, I, P, I, P], I),
    'eegan_nhwc_to_nchw': ([P, I, I, I, I, P, P], I),
    'eegan_fc_to_nhwc': ([P, I, I, I, I, P, I, P], I),
    'eegan_nhwc_to_fc': ([P, I, I, I, I, P, I, P], I),
    'eegan_maxpool3s2': ([P, I, I, I, I, I, P, I, P, P], I),
    'eegan_maxpool3s2_bwd': ([P, I, P, I, I, I, I, P, I, P], I),
    'eegan_avgpool3s1': ([P, I, I, I, I, I, P, I, P], I),
    'eegan_global_avgpool': ([P, I, I, I, I, P, I, P], I),
    'eegan_global_avgpool_bwd': ([P, I, I, I, I, P, I, P], I),
    'eegan_fill_f32': ([P, L, F, P], I),
    'eegan_stamp': ([P, P], I),
    'eegan_gemm_f32': ([P, L, L, P, L, L, P, L, I, I, I, P, I, F, F, P], I),
    'eegan_colsum_f32': ([P, L, I, I, P, I, P], I),
    'eegan_gemm_f32_grouped': ([C.POINTER(GemmDesc), I, P], I),
    'eegan_act_bwd_f32': ([P, P, L, I, F, P, P], I),
    'eegan_words_workspace': ([I, I, I, I], L),
    'eegan_words_sim': ([P, P, P, I, I, I, I, P, P, P, P], I),
    'eegan_words_sim_bwd': ([P, P, P, I, I, I, P, P, P, P, I, P], I),
    'eegan_sim_ce': ([P, I, P, P, P, P], I),
    'eegan_sim_ce_bwd': ([P, I, P, P, P, P, P], I),
    'eegan_gag_fwd_workspace': ([I, I], L),
    'eegan_gag_fwd': ([P, P, P, P, I, I, I, I, I, P, P, P, P], I),
    'eegan_gag_workspace': ([I, I, I, I, I], L),
    'eegan_gag_bwd': ([P, P, P, P, P, P, I, I, I, I, I, P, P, P, P, P], I),
    'eegan_sent_sim': ([P, P, I, I, I, P, P], I),
    'eegan_sent_sim_bwd': ([P, P, I, I, I, P, P, P, P, P, P], I),
    'eegan_dout_reduce': ([P, I, I, P, P], I),
    'eegan_dout_reduce_bwd': ([P, I, I, P, P, P], I),
    'eegan_bce_logits': ([P, P, I, P, P], I),
    'eegan_bce_logits_bwd': ([P, P, I, P, P, P], I),
    'eegan_gp_loss_workspace': ([I], L),
    'eegan_gp_loss': ([P, I, I, I, I, P, I, P, P, P, P], I),
    'eegan_gp_loss_bwd': ([P, I, I, I, I, P, I, P, P, P, I, P, P], I),
    'eegan_class_onehot': ([P, I, I, P, P, P], I),
    'eegan_attr_attn': ([P, P, P, I, I, I, F, P, P, P, P], I),
    'eegan_attr_attn_bwd': ([P, P, P, P, P, I, I, I, F, P, P, P, P], I),
    'eegan_adam': ([P, P, P, P, L, F, F, F, F, F, P, P], I),
    'eegan_adam_pack_blocks': ([I, I, I, I], L),
    'eegan_adam_range_blocks': ([L], L),
    'eegan_adam_pack': ([P, P, P, P, F, F, F, F, F, P, P, I, L, P], I),
    'eegan_embedding': ([P, L, P, I, P, P], I),
    'eegan_lstm_bidir': ([P, P, P, I, I, I, I, P, P, P], I),
    'eegan_fid_preprocess': ([P, I, I, I, I, I, P, P, P, I, P], I),
    'eegan_fid_samples_workspace': ([I, I, I], L),
    'eegan_fid_samples': ([P, I, I, I, I, I, I, P, P, I, P, P, I, P, P, P, I, P, P, P], I),
    'eegan_fid_stats_workspace': ([I], L),
    'eegan_fid_stats': ([P, I, I, P, P, P, P], I),
    'eegan_peer_region_bytes': ([I], L),
    'eegan_peer_alloc': ([L, P, P], I),
    'eegan_peer_open': ([P, P], I),
    'eegan_peer_close': ([P], I),
    'eegan_peer_free': ([P], I),
    'eegan_peer_allreduce_f64': ([P, I, I, I, I, P, P], I),
    'eegan_peer_set_wait': ([P, I], I),
    'eegan_peer_status': ([P, I, P], I),
    'eegan_pipe_workspace': ([I, I, I, I, P], L),
    'eegan_pipe_transform': ([P, P, I, I, I, P, P, I, P, P, P, I, P, P, P], I),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError('libeegan_hip.so not found at %s -- run __graft_entry__.build() '
                          '(make -C ee-gan_amd/csrc); there is no non-HIP fallback' % LIB_PATH)
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


LIB = _load()
ABI_VERSION = LIB.eegan_abi_version()
EXPECTED_ABI = 17
if ABI_VERSION != EXPECTED_ABI:
    raise ImportError('%s has ABI %d, these bindings need %d: rebuild (make -C ee-gan_amd/csrc)'
                      % (LIB_PATH, ABI_VERSION, EXPECTED_ABI))


class HipError(RuntimeError):
    pass


def _wrap(name):
    fn = getattr(LIB, name)
    if _SIGS[name][1] is not I or name == 'eegan_abi_version':
        return fn

    def call(*args):
        rc = fn(*args)
        if rc != 0:
            raise HipError('%s failed (%d): %s' % (name, rc, LIB.eegan_last_error().decode(errors='replace')))
        return rc
    call.__name__ = name
    return call


class _Ops:
    """`ops.conv_fwd(...)` -> checked call of `eegan_conv_fwd(...)`."""

    def __init__(self):
        for name in _SIGS:
            setattr(self, name[len('eegan_'):], _wrap(name))


ops = _Ops()


def exported_symbols():
    return sorted(_SIGS)
