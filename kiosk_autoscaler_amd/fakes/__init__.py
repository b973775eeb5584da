"""Test doubles: in-process Redis engine/client, RESP server, sentinel fakes.

See SURVEY §2.4 N8 and §4 ("Fakes and fixtures").
"""
from .engine import (BUSY_MESSAGE, FakeRedis, FakeStrictRedis, RedisEngine,
                     Session, glob_match)
from .server import RespServer
from .sentinel import SentinelCluster, FlakyRedis

__all__ = ['FakeRedis', 'FakeStrictRedis', 'RedisEngine', 'Session',
           'RespServer', 'SentinelCluster', 'FlakyRedis', 'BUSY_MESSAGE',
           'glob_match']
