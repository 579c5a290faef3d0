"""Namespace mirroring the reference's Clojure `jepsen.*` namespaces."""
