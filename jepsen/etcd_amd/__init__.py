"""jepsen.etcd_amd — MI355X-native linearizability checker for jepsen.etcd's
`register` workload (register.clj:102-119).

The hot path is `jepsen.independent/checker` around `checker/linearizable` with
the VersionedRegister model (register.clj:108-112).  This package is the host
side above the C ABI (include/lincheck.h): history preprocessing that mirrors
jepsen.independent / knossos history completion (`history`), and a Checker
with the reference's `check(test, history, opts)` shape (`checker`).
"""
from . import abi  # noqa: F401
