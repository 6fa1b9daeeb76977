"""AMQP 0-9-1 (RabbitMQ) messaging layer: wire codec, asyncio connection /
channels, and the job-level client (topology, shard fan-in, publisher,
reconnect)."""

from .client import Client, ConsumeError, Delivery, DeliveryMetadata
from .codec import AMQPError, Properties
from .connection import Channel, ChannelClosed, Connection, ConnectionClosed, Message, PublishNacked, PublishReturned

__all__ = ["Client", "Delivery", "DeliveryMetadata", "ConsumeError", "Connection", "Channel", "Message",
           "Properties", "AMQPError", "ConnectionClosed", "ChannelClosed", "PublishNacked",
           "PublishReturned"]
