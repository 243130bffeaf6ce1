"""Reference ops/basic_ops.py:4-6 (Identity), shared with the native trunk so that
`base_model.fc = Identity()` selects the fc-less trunk."""
from vcg_hip.nn import Identity  # noqa: F401
