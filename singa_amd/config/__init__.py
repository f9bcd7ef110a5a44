"""Reference-compatible configuration (ModelProto / ClusterProto / Topology)."""
from .schema import message_class, new, parse_text, read_text_file, to_text, enum_name  # noqa: F401
