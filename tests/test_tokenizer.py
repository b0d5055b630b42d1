"""Tokenizer / sampler / chat template / EosDetector behaviour (goldens ported from the reference's
src/tokenizer-test.cpp:122-303 and nn-cpu-ops-test.cpp softmax semantics)."""
import numpy as np
import pytest

EOS = 10000


def test_chat_template_detection(C):
    t = ("{% set loop_messages = messages %}{% for message in loop_messages %}{% set content = '<|start_header_id|>' "
         "+ message['role'] + '<|end_header_id|>\n\n'+ message['content'] | trim + '<|eot_id|>' %}")
    assert C.ChatTemplateGenerator("", t, "<eos>").type == "llama3"
    assert C.ChatTemplateGenerator("", "[INST] x", "<eos>").type == "llama2"
    assert C.ChatTemplateGenerator("", "x<｜Assistant｜>y", "<eos>").type == "deepSeek3"
    with pytest.raises(Exception):
        C.ChatTemplateGenerator("", "unknown", "<eos>")


def test_chat_templates_render(C):
    g = C.ChatTemplateGenerator("llama3", "", "<|eot_id|>")
    content, pub = g.generate([("system", "S"), ("user", "U")], True)
    assert content == (b"<|start_header_id|>system<|end_header_id|>\n\nS<|eot_id|>"
                       b"<|start_header_id|>user<|end_header_id|>\n\nU<|eot_id|>"
                       b"<|start_header_id|>assistant<|end_header_id|>\n\n")
    g2 = C.ChatTemplateGenerator("llama2", "", "</s>")
    content, _ = g2.generate([("system", "S"), ("user", "U")], True)
    assert content == b"[INST] <<SYS>>\nS\n<</SYS>>\n\nU [/INST]</s>"
    g3 = C.ChatTemplateGenerator("deepSeek3", "", "<eos>")
    content, pub = g3.generate([("user", "U")], True)
    assert pub == b"<think>\n" and content.endswith(b"<think>\n")


def _det(C, pieces, pad):
    return C.EosDetector([EOS, EOS + 1][:len(pieces)], pieces, pad, pad)


def test_eos_detector_with_padding(C):
    R = C.EosResult
    d = _det(C, ["<eos>", "<stop>"], 1)
    assert [d.append(1, "<"), d.append(2, "eo"), d.append(3, "s>")] == [R.MAYBE_EOS, R.MAYBE_EOS, R.EOS]
    assert d.get_delta() is None
    d.reset()
    assert [d.append(1, "<"), d.append(2, "stop"), d.append(3, "> ")] == [R.MAYBE_EOS, R.MAYBE_EOS, R.EOS]
    assert d.get_delta() is None
    d.reset()
    assert d.append(1, " ") == R.NOT_EOS and d.get_delta() == b" "
    d.reset()
    assert [d.append(1, "!<"), d.append(2, "eos"), d.append(3, "> ")] == [R.MAYBE_EOS, R.MAYBE_EOS, R.EOS]
    assert d.get_delta() == b"!"
    d.reset()
    assert [d.append(1, "<eo"), d.append(2, "s>XY")] == [R.MAYBE_EOS, R.NOT_EOS]
    assert d.get_delta() == b"<eos>XY"
    d.reset()
    assert [d.append(1, "<eo"), d.append(EOS, None)] == [R.MAYBE_EOS, R.EOS]
    assert d.get_delta() == b"<eo"
    d.reset()
    assert d.append(EOS, None) == R.EOS and d.get_delta() is None
    d.reset()
    assert d.append(1, "x") == R.NOT_EOS and d.get_delta() == b"x"
    d.reset()
    assert d.append(2, None) == R.NOT_EOS and d.get_delta() is None


def test_eos_detector_long_padding(C):
    R = C.EosResult
    d = C.EosDetector([EOS], ["|end|"], 5, 5)
    assert d.append(1, "lipsum") == R.NOT_EOS and d.get_delta() == b"lipsum"
    d.reset()
    assert d.append(1, "lorem") == R.NOT_EOS and d.get_delta() == b"lorem"
    d.reset()
    assert [d.append(1, "lorem|"), d.append(2, "enQ")] == [R.MAYBE_EOS, R.NOT_EOS]
    assert d.get_delta() == b"lorem|enQ"


def test_eos_detector_without_padding(C):
    R = C.EosResult
    d = C.EosDetector([EOS], ["<eos>"], 0, 0)
    assert [d.append(1, "<"), d.append(2, "eo"), d.append(3, "s>")] == [R.MAYBE_EOS, R.MAYBE_EOS, R.EOS]
    assert d.get_delta() is None
    d.reset()
    assert d.append(1, " <") == R.NOT_EOS and d.get_delta() == b" <"
    d.reset()
    assert [d.append(1, "<eos"), d.append(2, "> ")] == [R.MAYBE_EOS, R.NOT_EOS]
    assert d.get_delta() == b"<eos> "
    d.reset()
    assert d.append(EOS, None) == R.EOS and d.get_delta() is None
    d.reset()
    assert d.append(EOS, "\U0001F603") == R.EOS and d.get_delta() == "\U0001F603".encode()


def test_encode_decode_roundtrip(C, assets):
    t = C.Tokenizer(assets["tok"])
    text = "hello world, the end!"
    ids = t.encode(text, True, False)
    assert ids[0] == t.bos_id
    out = b""
    t.reset_decoder()
    for i in ids:
        p = t.decode(i)
        if p is not None:
            out += p
    assert out.decode() == text
    # merges happened: fewer tokens than bytes
    assert len(ids) - 1 < len(text.encode())


def test_encode_special_tokens(C, assets):
    t = C.Tokenizer(assets["tok"])
    ids = t.encode("<|start_header_id|>user<|end_header_id|>", False, True)
    assert ids[0] == t.bos_id + 2 and ids[-1] == t.bos_id + 3
    plain = t.encode("<|start_header_id|>", False, False)
    assert t.bos_id + 2 not in plain


def test_decode_utf8_stream(C, assets):
    t = C.Tokenizer(assets["tok"])
    emoji = "\U0001F603".encode()  # 4 bytes -> 4 single-byte tokens
    t.reset_decoder()
    outs = [t.decode(b) for b in emoji]
    assert outs[:3] == [None, None, None] and outs[3] == emoji
    # invalid continuation recovers with U+FFFD
    t.reset_decoder()
    assert t.decode(0xE2) is None
    assert t.decode(ord("a")) == "�a".encode()
    # eos flushes pending bytes
    t.reset_decoder()
    t.decode(0xF0)
    assert t.decode(t.eos_token_ids[0]) == b"\xf0"


def test_sampler(C):
    logits = np.array([0.1, 3.0, 0.2, 2.9], np.float32)
    assert C.Sampler(4, 0.0, 0.9, 1).sample(logits) == 1
    # seeded sampling is deterministic and covers high-probability tokens only with top-p
    s1, s2 = C.Sampler(4, 1.0, 0.5, 42), C.Sampler(4, 1.0, 0.5, 42)
    a = [s1.sample(logits) for _ in range(50)]
    b = [s2.sample(logits) for _ in range(50)]
    assert a == b and set(a) <= {1, 3}
    s3 = C.Sampler(4, 1.0, 1.0, 7)
    assert len({s3.sample(logits) for _ in range(400)}) == 4
