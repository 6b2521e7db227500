"""ctypes binding of liborbit_hip.so (C ABI: include/orbit_hip.h).

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7``
dependency resolves to the HIP runtime torch already loaded (one runtime, one set
of streams).  There is deliberately no fallback: if the library or a HIP device is
missing, every device entry point raises ``NativeUnavailable``.
"""
import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
# ORBIT_HIP_LIB selects an alternative build (kernel variants for tuning sweeps)
LIB_PATH = os.environ.get('ORBIT_HIP_LIB') or os.path.join(PKG, 'liborbit_hip.so')
ABI_VERSION = 19

c_i32, c_i64, c_dbl, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p

# numpy mirrors of the device tables (little-endian, C layout)
HALO_DTYPE = np.dtype([('cur_off', '<i8'), ('cur_cnt', '<i8'), ('prev_off', '<i8'),
                       ('prev_cnt', '<i8'), ('centre', '<f8', (3,)), ('bulk', '<f8', (3,)),
                       ('out_slot', '<i8'), ('reserved', '<i8')])
ITEM_DTYPE = np.dtype([('h0', '<i4'), ('h1', '<i4'), ('slot0', '<i4'), ('n_span', '<i4'),
                       ('scratch_off', '<i8'), ('n_pv', '<i8'), ('cur_off', '<i8'),
                       ('n_slots', '<i4'), ('reserved', '<i4')])

MODE = {'pericentric': 0, 'apocentric': 1}
STATUS_TABLE_OVERFLOW = 2
STATUS_PLAN = 4
STATUS_PART_OVERFLOW = 8
STATUS_LOOKBACK = 16
STATUS_PART_KEYS = 32


class StepArgs(ctypes.Structure):
    _fields_ = [('ids', c_vp), ('coords', c_vp), ('vels', c_vp), ('n_cur', c_i64),
                ('ids_prev', c_vp), ('rhat_prev', c_vp), ('meta_prev', c_vp), ('n_prev', c_i64),
                ('rhat_out', c_vp), ('meta_out', c_vp), ('angles_in', c_vp),
                ('halos', c_vp), ('n_halos', c_i32), ('items', c_vp), ('n_items', c_i32),
                ('H', c_dbl), ('one_plus_z', c_dbl), ('box', c_dbl * 3), ('n_box_dims', c_i32),
                ('coord_f64', c_i32), ('vel_f64', c_i32), ('dx_f64', c_i32), ('vb_f64', c_i32),
                ('wrap_f64', c_i32), ('id_bytes', c_i32), ('mode', c_i32), ('compare', c_i32),
                ('lds_entries', c_i32), ('lds_slots', c_i32),
                ('scratch_ids', c_vp), ('scratch_ang', c_vp), ('seg_count', c_vp),
                ('halo_count', c_vp), ('item_count', c_vp), ('status', c_vp),
                ('onthefly', c_i32), ('vr_f64', c_i32), ('angle_out', c_vp),
                ('matched_prev', c_vp), ('matched_cur', c_vp), ('vr_out', c_vp),
                ('n_global_items', c_i32), ('n_gchunk1', c_i32), ('n_gchunk2', c_i32),
                ('gchunk1', c_vp), ('gchunk2', c_vp), ('gtab', c_vp), ('gkeys', c_vp),
                ('gvals', c_vp), ('gtab_total', c_i64), ('scratch_pos', c_vp),
                ('n_parts', c_i32), ('part_kmax', c_i32), ('part_e', c_i32), ('part_slots', c_i32),
                ('prow', c_vp), ('gpart', c_vp),
                ('pkey_cur', c_vp), ('ppos_cur', c_vp), ('pmeta_cur', c_vp), ('prh_cur', c_vp),
                ('pkey_prev', c_vp), ('ppos_prev', c_vp), ('pmeta_prev', c_vp), ('prh_prev', c_vp),
                ('ikey', c_vp), ('ipos', c_vp), ('imeta', c_vp), ('irh', c_vp), ('icnt', c_vp),
                ('pcnt', c_vp), ('n_pcnt', c_i64), ('scratch_rk', c_vp), ('part_key4', c_i32),
                ('part_hi', ctypes.c_uint32), ('gchunk3', c_vp), ('n_gchunk3', c_i32),
                ('items_single', c_i32), ('direct', c_i32), ('lookback', c_vp),
                ('lb_epoch', c_i32), ('n_slots', c_i32), ('offsets_out', c_vp), ('out_ids', c_vp),
                ('out_ang', c_vp), ('out_pos', c_vp), ('total_out', c_vp),
                ('lb_spin_max', ctypes.c_uint32),
                ('reserved_abi16', c_i32)]


class UnbucketArgs(ctypes.Structure):
    _fields_ = [('bpos', c_vp), ('bmeta', c_vp), ('brh', c_vp), ('bcnt', c_vp), ('rows', c_vp),
                ('plist', c_vp), ('n_parts', c_i32), ('cap', c_i32), ('rhat_out', c_vp),
                ('meta_out', c_vp), ('td_f64', c_i32), ('reserved', c_i32)]


class CompactArgs(ctypes.Structure):
    _fields_ = [('halos', c_vp), ('n_halos', c_i32), ('items', c_vp), ('n_items', c_i32),
                ('ids_prev', c_vp), ('id_bytes', c_i32),
                ('scratch_ids', c_vp), ('scratch_ang', c_vp), ('seg_count', c_vp),
                ('halo_count', c_vp), ('item_count', c_vp), ('n_slots', c_i32),
                ('offsets_out', c_vp), ('out_ids', c_vp), ('out_ang', c_vp),
                ('total_out', c_vp), ('scratch_pos', c_vp), ('out_pos', c_vp),
                ('n_packed', c_i32), ('n_gchunks', c_i32), ('gchunks', c_vp),
                ('chunk_count', c_vp), ('scratch_rk', c_vp)]


class CollateArgs(ctypes.Structure):
    _fields_ = [('n_halos', c_i32), ('in_kind', c_i32), ('key_signed', c_i32),
                ('chunk_start', c_i32), ('lds_keys', c_i32), ('phases', c_i32),
                ('apsis_ids', c_vp), ('angles', c_vp), ('keep_lut', c_vp), ('src_off', c_vp),
                ('src_cnt', c_vp), ('new_base', c_vp), ('old_keys', c_vp), ('old_cnt', c_vp),
                ('old_off', c_vp), ('n_old', c_i64), ('n_new_cap', c_i64), ('w_keys', c_vp),
                ('w_cnt', c_vp), ('w_lb', c_vp), ('w_fp', c_vp), ('w_ulen', c_vp),
                ('w_found', c_vp), ('new_off', c_vp), ('new_keys', c_vp), ('new_cnt', c_vp),
                ('status', c_vp)]


class CentralArgs(ctypes.Structure):
    _fields_ = [('coords', c_vp), ('coord_f64', c_i32), ('dx_f64', c_i32),
                ('positions', c_vp), ('ids', c_vp), ('id_bytes', c_i32), ('n_halos', c_i32),
                ('offsets', c_vp), ('out_offsets', c_vp), ('n', c_i32), ('n_box_dims', c_i32),
                ('wrap_f64', c_i32 * 3), ('box', c_dbl * 3), ('half', c_dbl * 3),
                ('scratch', c_vp), ('out_ids', c_vp)]


class MainProgArgs(ctypes.Structure):
    _fields_ = [('halo_pids', c_vp), ('halo_kind', c_i32), ('n_halo_pids', c_i64),
                ('halo_offsets', c_vp), ('n_halos', c_i32), ('tracked', c_vp),
                ('tracked_kind', c_i32), ('n_tracked', c_i64), ('tracked_offsets', c_vp),
                ('n_blocks', c_i32), ('max_block', c_i32), ('tab_keys', c_vp), ('result', c_vp),
                ('status', c_vp)]


# include/orbit_post.h constants
ID_KIND = {np.dtype('int64'): 0, np.dtype('uint64'): 1, np.dtype('int32'): 2, np.dtype('uint32'): 3}
COLLATE_CHUNK = 4096
CENTRAL_MAX_N = 4096
POST_MISSING, POST_SENTINEL, POST_OVERFLOW, POST_BOUNDS = 1, 2, 4, 8

# every symbol include/orbit_hip.h and include/orbit_post.h declare: name -> (restype, argtypes)
SYMBOLS = {
    'oa_abi_version': (ctypes.c_int, []),
    'oa_build_info': (c_i32, [c_i32]),
    'oa_struct_size': (c_i64, [c_i32]),
    'oa_last_error': (ctypes.c_char_p, []),
    'oa_bulk_velocity': (ctypes.c_int, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp]),
    'oa_step': (ctypes.c_int, [ctypes.POINTER(StepArgs), c_vp]),
    'oa_step_lds_bytes': (c_i64, [c_i32, c_i32, c_i32]),
    'oa_part_lds_bytes': (c_i64, [c_i32, c_i32]),
    'oa_plan_items': (c_i64, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp,
                              c_i64, c_vp, c_vp]),
    'oa_max_lds_bytes': (c_i64, []),
    'oa_build_halos': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    'oa_debug_stamps': (c_i64, [c_vp, c_i64]),
    'oa_debug_part_stamps': (c_i64, [c_i32, c_vp, c_i64]),
    'oa_debug_central_stamps': (c_i64, [c_vp, c_i64]),
    'oa_compact': (ctypes.c_int, [ctypes.POINTER(CompactArgs), c_vp]),
    'oa_part_unbucket': (ctypes.c_int, [ctypes.POINTER(UnbucketArgs), c_vp]),
    'oa_match_workspace_bytes': (c_i64, [c_i64]),
    'oa_match_ids': (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp]),
    'oa_compare_pairs': (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                                        c_vp, c_vp, c_vp]),
    'oa_angle_add': (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    'oa_host_register': (ctypes.c_int, [c_vp, c_i64, ctypes.POINTER(c_vp)]),
    'oa_host_unregister': (ctypes.c_int, [c_vp]),
    'oa_stream_set_flag': (ctypes.c_int, [c_vp, c_vp, c_i64]),
    'oa_post_status': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    'oa_copy_bytes': (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp]),
    'oa_place_records': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp,
                                        c_vp]),
    # orbit_post.h
    'oa_post_struct_size': (c_i64, [c_i32]),
    'oa_collate_step': (ctypes.c_int, [ctypes.POINTER(CollateArgs), c_vp]),
    'oa_keys_to_ids': (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    'oa_retro_counts': (ctypes.c_int, [c_vp, c_i32, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp,
                                       c_vp, c_vp, c_vp]),
    'oa_central_ids': (ctypes.c_int, [ctypes.POINTER(CentralArgs), c_vp]),
    'oa_mainprog_workspace_bytes': (c_i64, [c_i64, c_i64]),
    'oa_main_progenitors': (ctypes.c_int, [ctypes.POINTER(MainProgArgs), c_vp]),
}


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    pass


_LIB = None


def load(require_device=False):
    """Load (once) and verify the native library; raise loudly if unusable."""
    global _LIB
    if _LIB is None:
        import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                'liborbit_hip.so not built: run `python -c "import __graft_entry__ as g; g.build()"`')
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SYMBOLS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.oa_abi_version() != ABI_VERSION:
            raise NativeUnavailable('liborbit_hip.so ABI %d != %d (stale build)'
                                    % (lib.oa_abi_version(), ABI_VERSION))
        sizes = {0: HALO_DTYPE.itemsize, 1: ITEM_DTYPE.itemsize,
                 2: ctypes.sizeof(StepArgs), 3: ctypes.sizeof(CompactArgs),
                 4: ctypes.sizeof(UnbucketArgs)}
        for k, v in sizes.items():
            if lib.oa_struct_size(k) != v:
                raise NativeUnavailable('ABI struct %d size mismatch: C %d, Python %d'
                                        % (k, lib.oa_struct_size(k), v))
        post = {0: ctypes.sizeof(CollateArgs), 1: ctypes.sizeof(CentralArgs),
                2: ctypes.sizeof(MainProgArgs)}
        for k, v in post.items():
            if lib.oa_post_struct_size(k) != v:
                raise NativeUnavailable('ABI post struct %d size mismatch: C %d, Python %d'
                                        % (k, lib.oa_post_struct_size(k), v))
        _LIB = lib
    if require_device:
        import torch
        if not torch.cuda.is_available():
            raise NativeUnavailable('no HIP device visible: the orbit kernels need an MI355X')
    return _LIB


def check(rc, what):
    if rc != 0:
        raise NativeError('%s failed (%d): %s' % (what, rc, _LIB.oa_last_error().decode()))
