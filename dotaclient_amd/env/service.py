"""gRPC transport for the DotaService contract (reference agent.py:880-881: grpclib client to localhost:13337).

``serve(service, port)`` exposes any object with ``reset_sync / observe_sync / act_sync`` (e.g. the
:class:`~dotaclient_amd.env.synthetic.SyntheticDotaService`, or an adapter around a real dotaservice) over gRPC with
the method paths ``/dotaservice.DotaService/{reset,observe,act}``; :class:`DotaServiceClient` is the matching
client with the same sync and async methods the actor uses. Built on ``grpcio`` generic handlers — no protoc-
generated stubs are needed (the message classes come from ``dotaclient_amd.protos``).
"""
from __future__ import annotations

import asyncio
from concurrent import futures
from typing import Optional

import grpc

from ..protos import SERVICE_NAME, pb

_METHODS = {
    'reset': (pb.GameConfig, pb.InitialObservation),
    'observe': (pb.ObserveConfig, pb.Observation),
    'act': (pb.Actions, pb.Empty),
}


def serve(service, port: int = 13337, host: str = '127.0.0.1', max_workers: int = 4) -> grpc.Server:
    handlers = {}
    for name, (req, resp) in _METHODS.items():
        fn = getattr(service, f'{name}_sync')
        handlers[name] = grpc.unary_unary_rpc_method_handler(
            (lambda f: (lambda request, context: f(request)))(fn),
            request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE_NAME, handlers),))
    bound = server.add_insecure_port(f'{host}:{port}')
    server.bound_port = bound
    server.start()
    return server


class DotaServiceClient:
    def __init__(self, host: str = '127.0.0.1', port: int = 13337, timeout: Optional[float] = 120.0):
        self.channel = grpc.insecure_channel(f'{host}:{port}')
        self.timeout = timeout
        self._calls = {}
        for name, (req, resp) in _METHODS.items():
            self._calls[name] = self.channel.unary_unary(f'/{SERVICE_NAME}/{name}',
                                                         request_serializer=req.SerializeToString,
                                                         response_deserializer=resp.FromString)

    # sync API (used by the batched Actor)
    def reset_sync(self, config):
        return self._calls['reset'](config, timeout=self.timeout)

    def observe_sync(self, observe_config):
        return self._calls['observe'](observe_config, timeout=self.timeout)

    def act_sync(self, actions):
        return self._calls['act'](actions, timeout=self.timeout)

    # async API (reference call style: `await dota_service.reset(config)`)
    async def reset(self, config):
        return await asyncio.get_running_loop().run_in_executor(None, self.reset_sync, config)

    async def observe(self, observe_config):
        return await asyncio.get_running_loop().run_in_executor(None, self.observe_sync, observe_config)

    async def act(self, actions):
        return await asyncio.get_running_loop().run_in_executor(None, self.act_sync, actions)

    def close(self):
        self.channel.close()
