"""backend.Backend gRPC contract: runtime-built message classes (`pb`), a servicer base with
generic handlers (`server.py`) and a persistent-channel client (`client.py`)."""
from __future__ import annotations

from google.protobuf import descriptor_pool, message_factory

from . import schema

_pool = descriptor_pool.DescriptorPool()
_fd = _pool.Add(schema.build_file_descriptor())


class _PB:
    """Namespace of message classes: pb.PredictOptions(...), pb.Reply(...), ..."""

    def __init__(self):
        for name in schema.MESSAGES:
            desc = _pool.FindMessageTypeByName(f"{schema.PACKAGE}.{name}")
            setattr(self, name, message_factory.GetMessageClass(desc))
        self.StatusState = {v: n for n, v in schema.ENUMS["StatusResponse.State"]}
        for n, v in schema.ENUMS["StatusResponse.State"]:
            setattr(self, f"STATE_{n}", v)


pb = _PB()
FULL_SERVICE = f"{schema.PACKAGE}.{schema.SERVICE}"
METHODS = {m[0]: m for m in schema.METHODS}
