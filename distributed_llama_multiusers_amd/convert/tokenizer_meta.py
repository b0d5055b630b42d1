"""Meta tokenizers -> `.t` (reference: converter/convert-tokenizer-llama3.py, convert-tokenizer-llama2.py).

  llama3 <tokenizer.model>   tiktoken rank file ("<base64 bytes> <rank>" lines) + the 256 Llama-3
                             special tokens, bos 128000, eos [128001, 128009], Llama-3 chat template
  llama2 <dir>               sentencepiece tokenizer.model with the Llama-2 [INST] chat template

usage: python -m distributed_llama_multiusers_amd.convert.tokenizer_meta {llama3|llama2} <path> [out_dir]
"""
from __future__ import annotations

import base64
import os
import sys

from ..utils.tfile import write_tokenizer

N_LLAMA3_SPECIAL = 256
LLAMA3_TEMPLATE = (
    "{% set loop_messages = messages %}{% for message in loop_messages %}{% set content = '<|start_header_id|>' + "
    "message['role'] + '<|end_header_id|>\n\n'+ message['content'] | trim + '<|eot_id|>' %}{% if loop.index0 == 0 %}"
    "{% set content = bos_token + content %}{% endif %}{{ content }}{% endfor %}{% if add_generation_prompt %}"
    "{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}{% endif %}")
LLAMA2_TEMPLATE = (
    "{% if messages[0]['role'] == 'system' %}{% set loop_messages = messages[1:] %}{% set system_message = "
    "messages[0]['content'] %}{% else %}{% set loop_messages = messages %}{% set system_message = false %}{% endif %}"
    "{% for message in loop_messages %}{% if loop.index0 == 0 and system_message != false %}{% set content = "
    "'<<SYS>>\\n' + system_message + '\\n<</SYS>>\\n\\n' + message['content'] %}{% else %}{% set content = "
    "message['content'] %}{% endif %}{% if message['role'] == 'user' %}{{ bos_token + '[INST] ' + content.strip() + "
    "' [/INST]' }}{% elif message['role'] == 'assistant' %}{{ ' '  + content.strip() + ' ' + eos_token }}{% endif %}"
    "{% endfor %}")


def llama3_special_tokens():
    named = ["<|begin_of_text|>", "<|end_of_text|>", "<|reserved_special_token_0|>", "<|reserved_special_token_1|>",
             "<|reserved_special_token_2|>", "<|reserved_special_token_3|>", "<|start_header_id|>",
             "<|end_header_id|>", "<|reserved_special_token_4|>", "<|eot_id|>"]
    return named + [f"<|reserved_special_token_{i}|>" for i in range(5, N_LLAMA3_SPECIAL - 5)]


def convert_llama3(rank_file: str, out_path: str) -> str:
    tokens, scores = [], []
    with open(rank_file) as f:
        for line in f:
            if not line.strip():
                continue
            b64, rank = line.split()
            tokens.append(base64.b64decode(b64))
            scores.append(-float(rank))
    n = len(tokens)
    for i, t in enumerate(llama3_special_tokens()):
        tokens.append(t.encode())
        scores.append(-float(n + i))
    bos = n  # 128000 for the real vocabulary
    write_tokenizer(out_path, tokens, scores, LLAMA3_TEMPLATE.encode(), bos, [bos + 1, bos + 9])
    return out_path


def convert_llama2(folder: str, out_path: str) -> str:
    from sentencepiece import SentencePieceProcessor
    sp = SentencePieceProcessor(model_file=os.path.join(folder, "tokenizer.model"))
    tokens = [sp.id_to_piece(i).replace("▁", " ").encode() for i in range(sp.vocab_size())]
    scores = [sp.get_score(i) for i in range(sp.vocab_size())]
    write_tokenizer(out_path, tokens, scores, LLAMA2_TEMPLATE.encode(), sp.bos_id(), [sp.eos_id()])
    return out_path


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2 or argv[0] not in ("llama3", "llama2"):
        print(__doc__)
        return 1
    out = os.path.join(argv[2] if len(argv) > 2 else ".", f"dllama_tokenizer_{argv[0]}.t")
    (convert_llama3 if argv[0] == "llama3" else convert_llama2)(argv[1], out)
    print(f"✅ Created {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
