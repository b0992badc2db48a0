"""ctypes binding of libsm_hip.so (include/sm_hip.h).

The product path is the HIP library; there is no CPU fallback. If the shared
object is missing or fails to load, importing this module raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SM_LIB_PATH") or os.path.join(HERE, "libsm_hip.so")  # override: A/B runs only
HEADER = os.path.join(os.path.dirname(HERE), "include", "sm_hip.h")


class SMError(RuntimeError):
    pass


class CGResult(ctypes.Structure):
    _fields_ = [("converged", ctypes.c_int), ("iterations", ctypes.c_int),
                ("residual", ctypes.c_double), ("phi_norm", ctypes.c_double)]


class HMCParams(ctypes.Structure):
    _fields_ = [("m0", ctypes.c_double), ("beta", ctypes.c_double), ("tau", ctypes.c_double),
                ("md_steps", ctypes.c_int), ("cg_tol", ctypes.c_double), ("cg_max_iter", ctypes.c_int),
                ("seed", ctypes.c_uint64), ("even_odd", ctypes.c_int)]


class HamiltonianTerms(ctypes.Structure):
    _fields_ = [("H", ctypes.c_double), ("kinetic", ctypes.c_double), ("gauge_action", ctypes.c_double),
                ("fermion", ctypes.c_double), ("sp", ctypes.c_double), ("cg_iterations", ctypes.c_int),
                ("cg_converged", ctypes.c_int)]


class HMCSummary(ctypes.Structure):
    _fields_ = [("Ep", ctypes.c_double), ("dEp", ctypes.c_double), ("gS", ctypes.c_double),
                ("dgS", ctypes.c_double), ("acceptance", ctypes.c_double), ("accepted", ctypes.c_long),
                ("trajectories", ctypes.c_long), ("cg_iterations", ctypes.c_long), ("cg_failures", ctypes.c_int),
                ("cg_link_bytes", ctypes.c_int)]


class HMCResult(ctypes.Structure):
    _fields_ = [("H_old", ctypes.c_double), ("H_new", ctypes.c_double), ("dH", ctypes.c_double),
                ("r", ctypes.c_double), ("accepted", ctypes.c_int), ("sp", ctypes.c_double),
                ("gauge_action", ctypes.c_double), ("cg_iterations", ctypes.c_long),
                ("cg_failures", ctypes.c_int)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (the HIP path has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    # Missing entry points are tolerated only when an A/B run says so
    # explicitly (SM_LIB_AB=1 with SM_LIB_PATH at an older build); any other
    # load, SM_LIB_PATH included, must export every entry point or fail here.
    ab_override = bool(os.environ.get("SM_LIB_PATH")) and os.environ.get("SM_LIB_AB") == "1"
    vp, ci, cd, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_long
    u64 = ctypes.c_uint64
    sig = {
        "sm_abi_version": ([], ci),
        "sm_last_error": ([], ctypes.c_char_p),
        "sm_shard_plan": ([ci, ci, ci, ctypes.POINTER(ci), ctypes.POINTER(ci)], ci),
        "sm_fill_gauge": ([u64, cd, ci, ci, ci, ci, ci, vp, vp], None),
        "sm_fill_spinor": ([u64, ci, ci, ci, ci, ci, vp, vp], None),
        "sm_conf_write": ([ctypes.c_char_p, ci, ci, vp, vp], ci),
        "sm_conf_read": ([ctypes.c_char_p, ci, ci, vp, vp], ci),
        "sm_comm_unique_id": ([vp, ci], ci),
        "sm_device_count": ([ctypes.POINTER(ci)], ci),
        "sm_create": ([ctypes.POINTER(vp), ci, ci, ci, ci, ci, vp], ci),
        "sm_create_hosted": ([ctypes.POINTER(vp), ci, ci, ci, ci, ci, vp], ci),
        "sm_create_loopback": ([ctypes.POINTER(vp), ci, ci, ci, vp], ci),
        "sm_peer_handle_bytes": ([], ci),
        "sm_create_peer": ([ctypes.POINTER(vp), ci, ci, ci, ci, ci, vp, ci], ci),
        "sm_peer_connect": ([vp, vp, ci], ci),
        "sm_create_peer_loopback": ([ctypes.POINTER(vp), ci, ci, ci], ci),
        "sm_peer_status": ([vp, ctypes.POINTER(ctypes.c_ulonglong)], ci),
        "sm_destroy": ([vp], ci),
        "sm_set_stream": ([vp, vp], ci),
        "sm_synchronize": ([vp], ci),
        "sm_tune": ([vp, ci, ci, ci, ci], ci),
        "sm_bench_stream": ([vp, ci, cl, vp, vp, vp, ci], ci),
        "sm_local_sites": ([vp, ctypes.POINTER(cl), ctypes.POINTER(ci), ctypes.POINTER(ci),
                            ctypes.POINTER(ci)], ci),
        "sm_upload_gauge": ([vp, vp, vp], ci),
        "sm_upload_gauge_dev": ([vp, vp], ci),
        "sm_dirac": ([vp, vp, vp, vp, vp, cd, ci], ci),
        "sm_ddag": ([vp, vp, vp, vp, vp, cd], ci),
        "sm_force": ([vp, vp, vp, vp, vp, vp, vp], ci),
        "sm_dot": ([vp, vp, vp, vp, vp, vp], ci),
        "sm_cg": ([vp, vp, vp, vp, vp, cd, cd, ci, ctypes.POINTER(CGResult)], ci),
        "sm_dirac_dev": ([vp, vp, vp, cd, ci], ci),
        "sm_ddag_dev": ([vp, vp, vp, cd], ci),
        "sm_force_dev": ([vp, vp, vp, vp], ci),
        "sm_dot_dev": ([vp, vp, vp, vp], ci),
        "sm_cg_dev": ([vp, vp, vp, cd, cd, ci, ctypes.POINTER(CGResult)], ci),
        "sm_cg_begin": ([vp, vp, vp, cd, cd], ci),
        "sm_cg_iterate": ([vp, ci], ci),
        "sm_cg_status": ([vp, ctypes.POINTER(CGResult)], ci),
        "sm_cg_finish": ([vp, ctypes.POINTER(CGResult)], ci),
        "sm_tune_cg": ([vp, ci, ci], ci),
        "sm_build_id": ([], ctypes.c_char_p),
        "sm_placement_report": ([vp, vp, ctypes.POINTER(ci), ctypes.POINTER(ci)], ci),
        "sm_set_placement_probe": ([ci], ci),
        "sm_get_placement_probe": ([], ci),
        "sm_placement_buffer_name": ([ci], ctypes.c_char_p),
        "sm_comm_info": ([vp, ctypes.POINTER(ci), ctypes.POINTER(ci), ctypes.POINTER(ci)], ci),
        "sm_cg_sums_in_pass": ([vp, ctypes.POINTER(ci)], ci),
        "sm_cg_link_codes": ([vp, ci, ctypes.POINTER(ci)], ci),
        "sm_cg_link_angles": ([vp, ci, ctypes.POINTER(ci)], ci),
        "sm_link_code_check": ([vp, vp, ctypes.POINTER(cd), ctypes.POINTER(ctypes.c_long)], ci),
        "sm_cg_link_bytes": ([vp, ctypes.POINTER(ci)], ci),
        "sm_tune_cg_geometry": ([vp, ci, ci], ci),
        "sm_tune_cg_strip": ([vp, ci, ci], ci),
        # gauge field / molecular dynamics / HMC
        "sm_download_gauge": ([vp, vp, vp], ci),
        "sm_fill_gauge_dev": ([vp, u64, cd], ci),
        "sm_plaquette": ([vp, cd, ctypes.POINTER(cd), ctypes.POINTER(cd), vp], ci),
        "sm_staples": ([vp, vp, vp], ci),
        "sm_gauge_force": ([vp, cd, vp, vp], ci),
        "sm_md_force": ([vp, ctypes.POINTER(HMCParams), vp, vp, vp, vp, ctypes.POINTER(CGResult)], ci),
        "sm_md_force_dev": ([vp, ctypes.POINTER(HMCParams), vp, vp, ctypes.POINTER(CGResult)], ci),
        "sm_leapfrog": ([vp, ctypes.POINTER(HMCParams), vp, vp, vp, vp, ctypes.POINTER(cl),
                         ctypes.POINTER(ci)], ci),
        "sm_leapfrog_dev": ([vp, ctypes.POINTER(HMCParams), vp, vp, ctypes.POINTER(cl), ctypes.POINTER(ci)], ci),
        "sm_hamiltonian": ([vp, ctypes.POINTER(HMCParams), vp, vp, vp, vp, ctypes.POINTER(HamiltonianTerms)], ci),
        "sm_hamiltonian_dev": ([vp, ctypes.POINTER(HMCParams), vp, vp, ctypes.POINTER(HamiltonianTerms)], ci),
        "sm_hmc_trajectory": ([vp, ctypes.POINTER(HMCParams), u64, ctypes.POINTER(HMCResult)], ci),
        "sm_quenched_trajectory": ([vp, ctypes.POINTER(HMCParams), u64], ci),
        "sm_hmc_run": ([vp, ctypes.POINTER(HMCParams), ci, u64, ci, ci, ci, ctypes.c_char_p,
                        ctypes.POINTER(HMCSummary), vp, vp], ci),
        "sm_jackknife_error": ([vp, ci, ci], cd),
        "sm_gather_gauge": ([vp, vp, vp], ci),
        "sm_eo_dhat": ([vp, ci, vp, vp, vp, vp, cd], ci),
        "sm_eo_cg": ([vp, vp, vp, vp, vp, cd, cd, ci, ctypes.POINTER(CGResult)], ci),
    }
    for name, (args, res) in sig.items():
        if ab_override and not hasattr(lib, name):
            continue  # an older build under an A/B override may predate newer entry points
        fn = getattr(lib, name)  # the product library must export every entry point
        fn.argtypes = args
        fn.restype = res
    return lib


lib = _load()


def check(rc):
    if rc != 0:
        raise SMError(f"sm_hip error {rc}: {lib.sm_last_error().decode(errors='replace')}")
    return rc
