"""CPU restatement of the reference's hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker (or, for the baseline, as the
thing timed on host cores).  The product path (jama16-retina-replication_amd/)
never imports it and fails loudly when libjr.so is missing.

Parity status: UNPINNED.  The reference's arithmetic lives in third-party
TensorFlow 1.x (version unpinned: "Tensorflow >= 1.4", README.md:15-23), which
is not installed here and cannot be (no network); the reference ships no
tests, golden vectors or fixtures.  The restatement
follows the reference call sites cited per function plus the TF semantics of
SURVEY.md Appendix B; it is cross-checked against independent formulations
(numpy fp64 direct loops vs torch-CPU ops, sklearn for ROC) in tests/.
"""
