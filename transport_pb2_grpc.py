"""Compat shim for the reference's generated gRPC module (fl_server.py:9, fl_client.py:9)."""
from crack_detection_federatedlearning_grpc_amd.fl.rpc import (TransportServiceServicer, TransportServiceStub,  # noqa: F401
                                                               add_TransportServiceServicer_to_server)
