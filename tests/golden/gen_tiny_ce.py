"""Writes tests/golden/tiny_ce/: a small seeded random-init BERT cross-encoder (BertForSequenceClassification,
one label) with the WordPiece vocab of tests/golden/tiny_bert.  Test model for the reranker parity test
(tests/test_gpu_reranker.py), whose oracle is Hugging Face's own pair encoding + forward on the CPU in
fp32.  Our own fixture model; no reference code involved (the reference reranker is an HTTP client)."""
import os
import shutil

import torch
from transformers import BertConfig, BertForSequenceClassification, BertTokenizer

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "tiny_ce")


def main():
    os.makedirs(OUT, exist_ok=True)
    shutil.copy(os.path.join(HERE, "tiny_bert", "vocab.txt"), os.path.join(OUT, "vocab.txt"))
    BertTokenizer(os.path.join(OUT, "vocab.txt"), do_lower_case=True).save_pretrained(OUT)
    n_vocab = sum(1 for _ in open(os.path.join(OUT, "vocab.txt")))
    cfg = BertConfig(vocab_size=n_vocab, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, max_position_embeddings=128, num_labels=1, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    torch.manual_seed(1)
    BertForSequenceClassification(cfg).save_pretrained(OUT, safe_serialization=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
