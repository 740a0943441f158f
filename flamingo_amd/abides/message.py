"""Message envelope of the ABIDES discrete-event simulation (message/Message.py surface).

A message is a free-form ``body`` dict passed by reference (no serialisation,
as in the reference, message/Message.py:12-45).  ``uniq`` is a global
creation counter used only to break ties between events due at the same time.
"""
from __future__ import annotations

import itertools
from enum import Enum, unique


@unique
class MessageType(Enum):
    MESSAGE = 1
    WAKEUP = 2

    def __lt__(self, other):
        return self.value < other.value


class Message:
    _counter = itertools.count()

    def __init__(self, body=None):
        self.body = body
        self.uniq = next(Message._counter)

    def __lt__(self, other):
        return self.uniq < other.uniq

    def __str__(self):
        return str(self.body)

    __repr__ = __str__
