"""Compat shim for the reference's generated module (fl_server.py:8, fl_client.py:8): the schema is built from
hand-written descriptors in crack_detection_federatedlearning_grpc_amd/fl/proto.py (protoc is unavailable)."""
from crack_detection_federatedlearning_grpc_amd.fl.proto import (DESCRIPTOR, FIN, NOT_WAIT, ON, TRAIN_DONE, TRAINING,  # noqa: F401
                                                                 WAIT, ReadyRep, ReadyReq, Scalar, State, UpdateRep,
                                                                 UpdateReq, VersionRep, VersionReq, transportRequest,
                                                                 transportResponse)
