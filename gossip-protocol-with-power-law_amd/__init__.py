"""MI355X-native gossip-propagation engine for the Seed/Peer protocol of
Sidharthshanu/Gossip-protocol-with-power-law.

Host side (Python): overlay builders and the seed registry mirror; hot path:
hand-written CDNA4 HIP kernels in csrc/, reached through the C-ABI of
include/gossip_capi.h (libgossip_hip.so, ctypes)."""
from . import bridge, degree, dist, overlay, peer, seed  # noqa: F401
from ._lib import GossipError, GossipLibraryError  # noqa: F401
from .engine import GossipEngine  # noqa: F401
from .overlay import CSR, NetworkBuilder, barabasi_albert, first3_overlay, powerlaw_join  # noqa: F401
from .seed import SeedRegistry  # noqa: F401
