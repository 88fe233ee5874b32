"""quill_amd — MI355X (gfx950) prover hot path for Quill (gio54321/quill-zkvm).

Host-side mirror of the reference's PCS / sumcheck surfaces over the C-ABI of
libquill_gpu.so (include/quill_gpu.h).  No CPU fallback: without the shared
library or a HIP device every entry point raises.
"""
from ._lib import LIB_PATH, QuillGpuError, lib  # noqa: F401
from .device import Device, DeviceVec, Srs  # noqa: F401
from .hyperplonk import (SumcheckProof, VirtualPolyExpr, VirtualPolynomialStore,  # noqa: F401
                         ZeroCheckProof)
from .pcs import (KZG, EvaluationClaim, KZGOpeningProof, MLEvalProof, g2_generator,  # noqa: F401
                  g2_mul, pairing)
from .transcript import Transcript  # noqa: F401
from .logup import (LookupMode, LookupProof, MultisetEqualityProof,  # noqa: F401
                    PermutationCheckProof, SetInclusionProof)
from .frontend import StateCell, TransitionCircuit, TransitionCircuitTarget  # noqa: F401
from .proof import (HyperPlonk, HyperPlonkProof, TracePK, TraceProof, TraceVK,  # noqa: F401
                    TraceWitness)
from .serialize import deserialize, serialize  # noqa: F401
