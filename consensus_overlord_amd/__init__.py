"""consensus_overlord_amd: MI355X-native BLS12-381 backend for the overlord `Crypto` trait of
cita-cloud/consensus_overlord. The arithmetic lives in libovhip.so (HIP,
gfx950); this package is the host-side mirror of the reference's ConsensusCrypto."""
from .crypto import (ConsensusCrypto, ConsensusError, Context, CryptoErr, DeviceError, Other,  # noqa: F401
                     raise_for)
from .vote import rlp_vote, vote_hash  # noqa: F401
