"""Shared document-dataset machinery: sample discovery, charset and class
maps, processor chain (reference: datasets/datapile_dataset.py:10-276 and
cassia_dataset.py:11-247, which duplicate this logic)."""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, List, Tuple

from torch.utils.data import Dataset

from gnn.data_generator import data_process
from gnn.utils.json_handler import read_json_file


class BaseDataset(Dataset):
    @classmethod
    def _from_config(cls, config: Dict[str, Any], **kwargs) -> "BaseDataset":
        return cls(config, **kwargs)


class DocumentDataset(BaseDataset):
    """Samples are JSON documents; each becomes a dict with the charset/class
    maps, then runs through the configured data_process chain."""

    def __init__(self, data_config: Dict[str, Any], **kwargs):
        self.logger = logging.getLogger(type(self).__module__)
        self.data_config = data_config
        self.list_samples = self._load_samples(kwargs.get("samples", None))
        self.num_samples = len(self.list_samples)
        self.charset = self._load_charset()
        self.char_to_id = {c: i for i, c in enumerate(self.charset)}
        self.id_to_char = {i: c for c, i in self.char_to_id.items()}
        self.classes, self.key_types = self._load_classes()
        self.class_to_id, self.id_to_class = self._map_class_to_id(self.classes, self.key_types)
        self.data_processors = self._load_data_processors()
        self.logger.info(f"Initialize {kwargs.get('data_type')} dataset, loading {self.num_samples} samples...")

    # -------------------------------------------------------------- samples
    def _load_samples(self, samples=None) -> List[Any]:
        if samples:
            return list(samples)
        paths = self.data_config.get("data_path") if hasattr(self.data_config, "get") else None
        if not paths:
            self.logger.error("Not found any dataset!")
            return []
        files: List[str] = []
        for folder in paths:
            if not os.path.exists(folder):
                self.logger.warning(f"Found invalid data path: {folder}")
                continue
            # one label file per stem (the reference keys files by stem)
            stems = {}
            for fn in sorted(os.listdir(folder)):
                stem, ext = os.path.splitext(fn)
                stems[stem] = ext
            files.extend(os.path.join(folder, stem + ext) for stem, ext in stems.items())
        return [read_json_file(f) for f in files]

    def _load_charset(self) -> List[str]:
        path = self.data_config.get("charset_path")
        if not path:
            raise ValueError("Not found any charset! (data_config.charset_path)")
        return read_json_file(path)["charset"]

    def _load_classes(self) -> Tuple[List[str], List[str]]:
        path = self.data_config.get("class_path")
        if not path:
            raise ValueError("Not found class list! (data_config.class_path)")
        return read_json_file(path)["classes"], list(self.data_config.get("key_types") or [])

    @staticmethod
    def _map_class_to_id(classes: List[str], key_types: List[str]):
        """class k, key type j -> index k*len(key_types) + j + 1 (0 = other)."""
        class_to_id: Dict[str, Dict[str, int]] = {}
        id_to_class: Dict[int, Tuple[str, str]] = {}
        for k, name in enumerate(classes):
            class_to_id[name] = {}
            for j, kt in enumerate(key_types):
                idx = k * len(key_types) + j + 1
                class_to_id[name][kt] = idx
                id_to_class[idx] = (name, kt)
        return class_to_id, id_to_class

    def _load_data_processors(self) -> list:
        if self.data_config.get("augmentations"):
            raise NotImplementedError("data augmentations are outside this engine's scope")
        procs = []
        for name, args in (self.data_config.get("data_process") or {}).items():
            proc = getattr(data_process, name, None)
            if proc is None:
                raise KeyError(f"Cannot find data processor {name}")
            procs.append(proc._from_config(args))
        return procs

    # ------------------------------------------------------------ protocol
    def _load_annotations(self, sample: Any) -> Dict[int, Dict[str, Any]]:
        raise NotImplementedError

    def __getitem__(self, index: int) -> Dict[str, Any]:
        sample = {
            "label": self._load_annotations(self.list_samples[index]),
            "charset": self.charset, "classes": self.classes, "char_to_id": self.char_to_id,
            "id_to_char": self.id_to_char, "class_to_id": self.class_to_id, "id_to_class": self.id_to_class,
        }
        for proc in self.data_processors:
            sample = proc(sample)
        return sample

    def __len__(self) -> int:
        return len(self.list_samples)
