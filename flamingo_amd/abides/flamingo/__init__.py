"""Flamingo protocol agents (agent/flamingo surface) backed by the MI355X engine."""
from .client_agent import SA_ClientAgent  # noqa: F401
from .service_agent import SA_ServiceAgent  # noqa: F401
