"""Offline wav -> wav speech dialogue (the caller above the drop-in boundary; reference bin/inference.py).

Same command line as the reference (bin/inference.py:29-41):
    python freeze-omni_amd/bin/inference.py --model_path DIR --llm_path DIR --input_wav in.wav --output_wav out.wav
and the same stage sequence (bin/inference.py:94-187): 'pre' with the default role, listen over
2560-sample chunks ('dialog_cl' forced after each chunk, as the reference does), reset the encoder
caches, 'dialog_ss', then 'dialog_cs' text steps until EOS or 128 tokens, speaking each sentence as
soon as it ends (suffixes bin/inference.py:166-175; the "." after a digit does not end one).

Differences from the reference script, all on the host side of the boundary:
  * wav I/O uses the stdlib `wave` module (soundfile is not in this image); input is 16-bit PCM
    (or 32-bit float via scipy.io.wavfile), scaled to [-1, 1) as soundfile does.
  * input not at 16 kHz is resampled with scipy.signal.resample_poly instead of
    torchaudio.transforms.Resample (torchaudio is not in this image): resampled inputs are not
    bit-identical to the reference's.
  * the output is written as 16-bit PCM at 24 kHz (the reference writes soundfile's default subtype
    for float input, PCM_16 for .wav).
Fbank, encoder, LLM, text decode, speech decoder and vocoder all run on the MI355X engine.
"""
import argparse
import math
import os
import sys
import wave

import numpy as np
import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from models.audio_processor import audioEncoderProcessor  # noqa: E402
from models.decoder.llm2tts import llm2TTS  # noqa: E402
from models.pipeline import inferencePipeline  # noqa: E402

SUFFIXES = ("。", "：", "？", "！", ".", "?", "!", "\n")   # bin/inference.py:166
MAX_TEXT_TOKENS = 128                                       # bin/inference.py:153


def get_args(argv=None):
    p = argparse.ArgumentParser(description="Freeze-Omni (MI355X)")
    p.add_argument("--model_path", required=True, help="model_path to load")
    p.add_argument("--llm_path", required=True, help="llm_path to load")
    p.add_argument("--top_k", type=int, default=5)
    p.add_argument("--top_p", type=float, default=0.8)
    p.add_argument("--temperature", type=float, default=0.7)
    p.add_argument("--input_wav", required=True, help="input wav")
    p.add_argument("--output_wav", required=True, help="output wav")
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--role", default="You are a helpful assistant.")
    p.add_argument("--max_text_tokens", type=int, default=MAX_TEXT_TOKENS)
    args = p.parse_args(argv)
    print(args)
    return args


def read_wav(path):
    """-> (float64 samples in [-1, 1), sample rate); mono (the first channel of a multi-channel file)."""
    try:
        with wave.open(path, "rb") as f:
            fs, ch, sw, n = f.getframerate(), f.getnchannels(), f.getsampwidth(), f.getnframes()
            raw = f.readframes(n)
        if sw != 2:
            raise ValueError(f"{path}: {8 * sw}-bit PCM; 16-bit PCM or 32-bit float expected")
        x = np.frombuffer(raw, dtype="<i2").reshape(-1, ch)[:, 0].astype(np.float64) / 32768.0
        return x, fs
    except wave.Error:   # IEEE float wav (format 3) is not readable by `wave`
        from scipy.io import wavfile
        fs, x = wavfile.read(path)
        x = np.asarray(x)
        if x.ndim > 1:
            x = x[:, 0]
        if x.dtype.kind == "f":
            return x.astype(np.float64), fs
        raise


def write_wav(path, pcm, fs=24000):
    q = np.clip(np.round(np.asarray(pcm, dtype=np.float64) * 32768.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(fs)
        f.writeframes(q.tobytes())


def resample_to_16k(x, fs):
    if fs == 16000:
        return x
    from scipy.signal import resample_poly
    g = math.gcd(int(fs), 16000)
    return resample_poly(x, 16000 // g, int(fs) // g)


def decoder(cur_hidden_state, pipeline, cur_text, tts, codec_chunk_size, codec_padding_size, decoder_topk, wav):
    """bin/inference.py:82-92: speak one sentence from its LLM hidden states and normalised text."""
    idim = tts.model.idim
    hidden = torch.cat(cur_hidden_state).reshape(-1, idim).unsqueeze(0)
    text = pipeline.post_process(cur_text)
    print("Synthesis: ", [text])
    emb = pipeline.model.llm_decoder.model.embed_tokens(pipeline.model.tokenizer.encode(text))
    for seg in tts.run(emb.reshape(-1, idim).unsqueeze(0), decoder_topk, hidden, codec_chunk_size,
                       codec_padding_size):
        wav.append(seg)


def inference(pipeline, audio_processor, tts, configs):
    """bin/inference.py:94-187. Returns (whole_text, pcm float32 numpy at 24 kHz)."""
    x, fs = read_wav(configs.input_wav)
    x = resample_to_16k(x, fs)
    codec_chunk_size, codec_padding_size, decoder_topk = 40, 10, 2   # bin/inference.py:113-115

    outputs = pipeline.speech_dialogue(None, stat="pre", role=getattr(configs, "role", None)
                                       or "You are a helpful assistant.")
    chunk = audio_processor.get_chunk_size()
    pcm = np.zeros(math.ceil(x.shape[0] / chunk) * chunk)
    pcm[:x.shape[0]] = x
    for i in range(0, pcm.shape[0], chunk):
        fb = audio_processor.process(torch.from_numpy(pcm[i:i + chunk]))
        outputs = pipeline.speech_dialogue(fb, **outputs)
        outputs["stat"] = "dialog_cl"
    audio_processor.reset()
    outputs.update(adapter_cache=None, encoder_cache=None, pe_index=0, stat="dialog_ss")

    outputs = pipeline.speech_dialogue(None, **outputs)
    cur_hidden_state = [outputs["hidden_state"]]
    whole_text = last_text = cur_text = ""
    wav = []
    limit = getattr(configs, "max_text_tokens", MAX_TEXT_TOKENS)
    while len(outputs["past_tokens"]) <= limit:
        del outputs["text"], outputs["hidden_state"]
        outputs = pipeline.speech_dialogue(None, **outputs)
        if outputs["stat"] == "dialog_cs":
            cur_hidden_state.append(outputs["hidden_state"])
            new = outputs["text"][len(last_text):]
            whole_text += new
            cur_text += new
            if new.endswith(SUFFIXES) and not (new.endswith(".") and last_text and last_text[-1].isdigit()):
                if cur_hidden_state:
                    decoder(cur_hidden_state, pipeline, cur_text, tts, codec_chunk_size, codec_padding_size,
                            decoder_topk, wav)
                    cur_hidden_state = []
                cur_text = ""
        if outputs["stat"] == "dialog_sl":
            break
        last_text = outputs["text"]
    if cur_hidden_state:
        decoder(cur_hidden_state, pipeline, cur_text, tts, codec_chunk_size, codec_padding_size, decoder_topk,
                wav)
    out = torch.cat([w.reshape(-1) for w in wav]).float().cpu().numpy() if wav else np.zeros(0, np.float32)
    write_wav(configs.output_wav, out, 24000)
    if hasattr(outputs["past_key_values"], "free"):
        outputs["past_key_values"].free()
    print(whole_text)
    return whole_text, out


def main(argv=None):
    configs = get_args(argv)
    pipeline = inferencePipeline(configs)
    tts = llm2TTS(configs.model_path, device=configs.device)
    audio_processor = audioEncoderProcessor(device=configs.device)
    return inference(pipeline, audio_processor, tts, configs)


if __name__ == "__main__":
    main()
