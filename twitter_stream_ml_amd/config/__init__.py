"""Configuration: HOCON-subset loader and the twtml-spark CLI."""
from .hocon import (Config, ConfigError, ConfigFactory, clear_property, get_property,
                    load_java_opts, parse_hocon, set_property, system_properties)
from .arguments import ConfArguments, MasterSpec, SparkConf, parse_master

__all__ = [
    "Config", "ConfigError", "ConfigFactory", "ConfArguments", "MasterSpec", "SparkConf",
    "clear_property", "get_property", "load_java_opts", "parse_hocon", "parse_master",
    "set_property", "system_properties",
]
