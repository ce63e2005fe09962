"""ctypes binding of libsafelife_hip.so -- the C ABI declared in include/safelife_hip.h.

The product path has no CPU fallback: if the HIP library is missing, or no GPU is
visible, every entry point raises.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "_native", "libsafelife_hip.so")
LIB_PATH = os.environ.get("SAFELIFE_HIP_LIB") or _DEFAULT_LIB
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

SL_OK, SL_EINVAL, SL_EHIP, SL_ETOOBIG = 0, -1, -2, -3
SL_RNG_STREAM, SL_RNG_PHILOX = 0, 1
SL_KERNEL_AUTO, SL_KERNEL_GENERIC, SL_KERNEL_FAST = 0, 1, 2
SL_STREAM_ERR_RANGE, SL_STREAM_ERR_THRESHOLD = 1, 2
SL_BOARD_AUTO, SL_BOARD_UINT16 = 0, 1
SL_MAX_EXITS = 8
SL_BONUS_PERIOD_MAX = 16
SL_OBS_NONE, SL_OBS_PACKED, SL_OBS_CHANNELS, SL_OBS_CHANNELS_U8 = 0, 1, 2, 3
SL_OBS_CHANNELS_F32, SL_OBS_CHANNELS_BF16 = 4, 5

_ERRORS = {SL_EINVAL: "invalid argument / shape", SL_EHIP: "HIP launch error",
           SL_ETOOBIG: "board too large for this kernel"}

vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
u32 = ctypes.c_uint32
u64 = ctypes.c_uint64
f32 = ctypes.c_float
f64 = ctypes.c_double


class EnvState(ctypes.Structure):
    _fields_ = [("B", i64), ("H", i32), ("W", i32),
                ("board", vp), ("goals", vp), ("start_board", vp),
                ("agent_x", vp), ("agent_y", vp), ("orientation", vp),
                ("game_over", vp), ("episode_length", vp), ("episode_reward", vp),
                ("old_points", vp), ("baseline", vp), ("score", vp), ("possible", vp),
                ("side_effect", vp), ("spawn_prob", vp), ("min_performance", vp),
                ("prior_x", vp), ("prior_y", vp), ("prior_len", vp), ("prior_head", vp),
                ("exit_count", vp), ("exit_y", vp), ("exit_x", vp),
                ("level_index", vp), ("episodes", vp), ("num_steps", vp),
                ("spawn_flags", vp), ("start_roll", vp), ("planes", vp), ("planes_ok", vp),
                ("elig_planes", vp), ("board_planes", vp), ("board_zero", u32),
                ("planes_live", i32)]


class LevelPool(ctypes.Structure):
    _fields_ = [("K", i32), ("H", i32), ("W", i32),
                ("board", vp), ("goals", vp), ("agent_x", vp), ("agent_y", vp),
                ("orientation", vp), ("spawn_prob", vp), ("min_performance", vp),
                ("board_planes", vp), ("goal_planes", vp)]


class EnvCfg(ctypes.Structure):
    _fields_ = [("time_limit", i32), ("auto_reset", i32),
                ("can_toggle_powers", i32), ("can_toggle_colors", i32),
                ("penalty_coef", f64), ("wrapper_min_performance", f64),
                ("bonus_table", vp), ("bonus_len", i32), ("bonus_period", i32),
                ("rng_mode", i32), ("seed", u64), ("step", u32), ("env0", u32),
                ("draws", vp), ("n_draws", i64), ("stream_pos", vp), ("scratch", vp),
                ("level_mode", i32), ("n_total_envs", i32), ("augment_roll", i32),
                ("ev_begin", vp), ("ev_end", vp), ("kernel", i32),
                ("obs_out", vp), ("obs_mode", i32), ("obs_vh", i32), ("obs_vw", i32),
                ("obs_remove_white", i32), ("obs_nch", i32), ("obs_channels", i32 * 16),
                ("capture", vp), ("stream_phase", i32), ("stream_base", vp), ("mt", vp),
                ("board_mode", i32)]


class MT19937(ctypes.Structure):
    _fields_ = [("n_chains", i32), ("rounds", i32), ("ring_draws", i64), ("ring", vp),
                ("chains", vp), ("prefix", vp), ("polys", vp), ("ctl", vp),
                ("ahead_stream", vp), ("ev_fill", vp), ("ev_ahead", vp),
                ("ahead_pending", i32), ("bit_ring", i32), ("bits_thr", f64)]


class Capture(ctypes.Structure):
    _fields_ = [("n", i32), ("env", vp), ("board", vp), ("goals", vp), ("orientation", vp),
                ("flags", vp), ("reset_board", vp), ("reset_goals", vp),
                ("reset_orientation", vp)]


_lib = None


class HipUnavailable(RuntimeError):
    pass


def build(force=False):
    """Compile the HIP library in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", CSRC])


def lib():
    """Load the HIP library; raise if it is missing (there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipUnavailable(
            "libsafelife_hip.so not built (%s); run `make -C %s` -- the SafeLife HIP "
            "path has no CPU fallback" % (LIB_PATH, CSRC))
    L = ctypes.CDLL(LIB_PATH)
    L.sl_version.restype = ctypes.c_char_p
    L.sl_build_id.restype = ctypes.c_char_p
    L.sl_device_arch.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.sl_advance.argtypes = [vp, vp, i64, ctypes.c_int, ctypes.c_int, vp, f32, ctypes.c_int,
                             u64, u32, u32, u32, vp, vp, vp]
    L.sl_count_eligible.argtypes = [vp, vp, i64, ctypes.c_int, ctypes.c_int, vp]
    L.sl_exclusive_scan_i64.argtypes = [vp, vp, i64, vp, vp, vp]
    if hasattr(L, "sl_host_advance") or LIB_PATH == _DEFAULT_LIB:
        L.sl_host_advance.argtypes = [vp, vp, i64, i64, f32, vp, i64]
        L.sl_host_advance.restype = i64
    L.sl_copy16.argtypes = [vp, vp, i64, vp]
    L.sl_env_step.argtypes = [ctypes.POINTER(EnvState), ctypes.POINTER(LevelPool), vp,
                              ctypes.POINTER(EnvCfg), vp, vp, vp, vp, vp, vp]
    L.sl_env_reset.argtypes = [ctypes.POINTER(EnvState), ctypes.POINTER(LevelPool), vp,
                               ctypes.POINTER(EnvCfg), vp]
    L.sl_level_pool_prepare.argtypes = [ctypes.POINTER(LevelPool), vp]
    L.sl_side_effect_workspace.argtypes = [i64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(i64)]
    L.sl_side_effect_densities.argtypes = [vp, vp, vp, vp, vp, i64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, u64, u32, vp, vp,
                                           ctypes.c_int, vp, vp, vp, vp, vp, vp, i64, vp]
    L.sl_env_obs.argtypes = [ctypes.POINTER(EnvState), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, vp, ctypes.c_int, vp, vp]
    L.sl_sample_actions.argtypes = [vp, ctypes.c_int, i64, ctypes.c_int, i64, ctypes.c_int, vp,
                                    u64, u32, u32, f64, vp, vp, vp]
    L.sl_gae.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, i64, f64, vp, vp, vp]
    L.sl_emd_cells.argtypes = [vp, vp, vp, vp, i64, vp, ctypes.c_int, ctypes.c_int, f64,
                               ctypes.POINTER(f64)]
    game = {"sl_env_action": [ctypes.POINTER(EnvState), vp, ctypes.c_int, ctypes.c_int, vp, vp],
            "sl_env_advance": [ctypes.POINTER(EnvState), ctypes.POINTER(EnvCfg), vp],
            "sl_env_rescore": [ctypes.POINTER(EnvState), vp, vp],
            "sl_env_exit_colors": [ctypes.POINTER(EnvState), ctypes.c_int, vp],
            "sl_env_board_sync": [ctypes.POINTER(EnvState), vp]}
    for name, args in game.items():
        # (an A/B build of an older revision, SAFELIFE_HIP_LIB, may lack these)
        if hasattr(L, name) or LIB_PATH == _DEFAULT_LIB:
            getattr(L, name).argtypes = args
            getattr(L, name).restype = ctypes.c_int
    mt = {"sl_mt19937_seed": [ctypes.POINTER(MT19937), u32, i64, vp],
          "sl_mt19937_fill": [ctypes.POINTER(MT19937), vp, vp, vp, vp],
          "sl_mt19937_lookahead": [ctypes.POINTER(MT19937), vp],
          "sl_mt19937_release": [ctypes.POINTER(MT19937)],
          "sl_mt19937_host_window": [u32, vp],
          "sl_mt19937_host_jump_poly": [u64, vp],
          "sl_mt19937_host_jump": [vp, vp, vp],
          "sl_mt19937_host_draws": [vp, i64, vp]}
    for name, args in mt.items():
        if hasattr(L, name) or LIB_PATH == _DEFAULT_LIB:
            getattr(L, name).argtypes = args
            getattr(L, name).restype = ctypes.c_int
    L.sl_event_create.argtypes = [ctypes.POINTER(vp)]
    L.sl_event_destroy.argtypes = [vp]
    L.sl_event_elapsed_ms.argtypes = [vp, vp, ctypes.POINTER(f32)]
    for name in ("sl_event_create", "sl_event_destroy", "sl_event_elapsed_ms", "sl_device_arch", "sl_advance", "sl_count_eligible", "sl_exclusive_scan_i64",
                 "sl_env_step", "sl_env_reset", "sl_env_obs", "sl_level_pool_prepare",
                 "sl_side_effect_workspace", "sl_side_effect_densities",
                 "sl_sample_actions", "sl_gae", "sl_emd_cells", "sl_copy16"):
        getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def check(rc, what):
    if rc != SL_OK:
        raise RuntimeError("%s failed: %s (code %d)" % (what, _ERRORS.get(rc, "?"), rc))


def require_device(device=None):
    """The torch device to run on; raises when no GPU is visible."""
    import torch
    if not torch.cuda.is_available():
        raise HipUnavailable("no ROCm GPU visible: the SafeLife HIP path needs an MI355X "
                             "(gfx950); there is no CPU fallback")
    lib()
    return torch.device(device if device is not None else "cuda:%d" % torch.cuda.current_device())


def stream_ptr(device):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def build_id():
    """Hash of the sources the loaded library was built from (Makefile BUILD_ID)."""
    return lib().sl_build_id().decode()
