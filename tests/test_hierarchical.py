"""HierarchicalMarkdownSplitter (hiprag.rag.chunker) against tests/golden/hierarchical.json, produced by the
REFERENCE's own splitter (utu/rag/knowledge_builder/chunker.py:124-349; tests/golden/gen_hierarchical.py):
45 markdown texts x 5 chunk configs, every chunk list equal."""
import json
import os

import pytest

from hiprag.rag import HierarchicalMarkdownSplitter
from hiprag.rag.config import ChunkingConfig


@pytest.fixture(scope="module")
def golden(golden_dir):
    return json.load(open(os.path.join(golden_dir, "hierarchical.json")))


def test_hierarchical_splitter_matches_reference(golden):
    for case in golden["cases"]:
        sp = HierarchicalMarkdownSplitter(ChunkingConfig(strategy="hierarchical", chunk_size=case["chunk_size"],
                                                         chunk_overlap=case["chunk_overlap"]))
        for text, want in zip(golden["texts"], case["chunks"]):
            assert sp.split_text(text) == want, (case["chunk_size"], case["chunk_overlap"], text[:80])
