"""Hand-written gRPC glue for ``TransportService.transport`` (the reference's generated transport_pb2_grpc).

One bidirectional-streaming method (fl_server.py:209-212, fl_client.py:85 ``stub.transport(generator)``).
"""
from __future__ import annotations

import grpc

from . import proto as P


def channel_options(max_message_mb: int = 512):
    n = int(max_message_mb) * 1024 * 1024
    # the reference misspells the send option ('grcp.', fl_server.py:215); both limits are applied here
    return [("grpc.max_receive_message_length", n), ("grpc.max_send_message_length", n)]


class TransportServiceStub:
    def __init__(self, channel: grpc.Channel):
        self.transport = channel.stream_stream(
            P.METHOD,
            request_serializer=P.transportRequest.SerializeToString,
            response_deserializer=P.transportResponse.FromString,
        )


class TransportServiceServicer:
    def transport(self, request_iterator, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method not implemented!")
        raise NotImplementedError("Method not implemented!")


def add_TransportServiceServicer_to_server(servicer: TransportServiceServicer, server: grpc.Server) -> None:
    handlers = {
        "transport": grpc.stream_stream_rpc_method_handler(
            servicer.transport,
            request_deserializer=P.transportRequest.FromString,
            response_serializer=P.transportResponse.SerializeToString,
        )
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(P.SERVICE, handlers),))
