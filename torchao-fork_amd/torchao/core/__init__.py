from .config import AOBaseConfig

__all__ = ["AOBaseConfig"]
