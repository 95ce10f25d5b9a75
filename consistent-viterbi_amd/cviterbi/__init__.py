"""cviterbi -- MI355X-native Viterbi decode path behind the consistent-viterbi solver API.

Host mirror of the reference's hmm::HMM and viterbi_solver interfaces over the C ABI
in include/cviterbi.h (libcviterbi.so: hand-written gfx950 HIP kernels).
"""
from ._lib import CVError, EXPORTS, LIB_PATH  # noqa: F401
from .hmm import HMM, tuning_keys  # noqa: F401
from .decode import (constrained_pairs, constrained_partials, constrained_select, decode, decode_batch, decode_batch_device, decode_constrained_device, decode_constrained_exchange,  # noqa: F401
                     decode_constrained, decode_forced_components, decode_superseq_cp, device_memory, last_suffix_traced, last_superseq_stats, last_timing, timing_begin,
                     timing_end)
from .fit import fit_mle, fit_train  # noqa: F401
from .solver import (Constraints, GpuSolver, Solver, SuperSequence, load_sequences, load_tags,  # noqa: F401
                     write_output)
