"""ABIDES discrete-event surface kept from the reference (Kernel.py, agent/, message/, model/).

The simulation runs on the host in one Python process, exactly as in the
reference; only the Flamingo agents' vector arithmetic goes to the GPU.
"""
from .agent import Agent  # noqa: F401
from .kernel import Kernel  # noqa: F401
from .latency import LatencyModel  # noqa: F401
from .message import Message, MessageType  # noqa: F401
