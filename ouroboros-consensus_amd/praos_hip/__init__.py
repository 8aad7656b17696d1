"""praos_hip: host-side binding of libpraos_hip.so (MI355X batch validator for
Ouroboros Praos header crypto).  See include/praos_hip.h for the C ABI."""
from .abi import Context, Params, load, params, LIB_PATH, HEADER_PATH  # noqa: F401
from . import abi, fixed  # noqa: F401
