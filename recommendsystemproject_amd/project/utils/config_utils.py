"""YAML config I/O — same functions as project/utils/config_utils.py (load_config/file_loader
with yaml.safe_load, save_config with safe_dump)."""
import os

import yaml


def load_config(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f'Config file not found at: {path}')
    with open(path, 'r', encoding='utf-8') as f:
        return yaml.safe_load(f)


def save_config(config_dict, path):
    d = os.path.dirname(path)
    if d and not os.path.exists(d):
        os.makedirs(d, exist_ok=True)
    with open(path, 'w', encoding='utf-8') as f:
        yaml.safe_dump(config_dict, f, default_flow_style=False, sort_keys=False, allow_unicode=True)
    print(f'Configuration saved to {path}')


file_loader = load_config
