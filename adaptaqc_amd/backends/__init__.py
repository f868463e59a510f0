from .aer_mps_backend import AerMPSBackend, HipMPSBackend, mps_sim_with_args  # noqa: F401
from .aer_sv_backend import AerSVBackend, HipSVBackend  # noqa: F401
from .aqc_backend import AQCBackend  # noqa: F401
