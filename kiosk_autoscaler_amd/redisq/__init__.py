"""In-tree Redis access layer: RESP2 codec, client, sentinel-aware retry proxy.

Replaces redis-py (unavailable here) under the reference's L1 layer
(``autoscaler/redis.py``); see SURVEY §1.1 L1 and §2.4 N7.
"""
from . import exceptions
from .client import Pipeline, Redis, StrictRedis
from .connection import Connection, ConnectionPool
from .failover import REDIS_READONLY_COMMANDS, RedisClient
from .resp import RespParser, encode_command

__all__ = ['exceptions', 'Redis', 'StrictRedis', 'Pipeline', 'Connection',
           'ConnectionPool', 'RedisClient', 'REDIS_READONLY_COMMANDS',
           'RespParser', 'encode_command']
