// hr_text.cpp -- host-side text kernel of the offline tokenizer (hiprag.rag.rocm_embedder.HashWordTokenizer):
// the lower-cased \w+ | [^\w\s] word split of ASCII texts and the crc32 hash of every word into
// [first_id, first_id + span), in one pass over the bytes.  Ingest feeds it every chunk it embeds; the
// Python restatement (re.findall + zlib.crc32 per word) cost ~40 % of the ingest host time.
// Same ids as the Python path for ASCII input (Python's str-pattern classes restricted to ASCII:
// \w = [0-9A-Za-z_], \s = [\t\n\v\f\r\x1c-\x1f ]); non-ASCII texts stay on the Python path.
#include <cstdint>

#include "../../include/hiprag.h"

namespace {

struct Crc32 {  // zlib's crc32 (reflected 0xEDB88320), table-driven
    uint32_t t[256];
    Crc32() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[i] = c;
        }
    }
};
const Crc32 kCrc;

inline uint8_t lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }
inline bool is_word(uint8_t c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
}
inline bool is_space(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }

}  // namespace

extern "C" int hr_hash_words(const char* text, const int64_t* offsets, int64_t n_texts, int64_t first_id, int64_t span,
                             int64_t cap, int64_t cls_id, int64_t sep_id, int64_t* ids_out, int64_t ids_cap,
                             int64_t* lengths_out) {
    if (n_texts < 0 || span <= 0 || (n_texts > 0 && (!offsets || !lengths_out)) || ids_cap < 0) return HR_E_INVALID;
    const bool special = cls_id >= 0 && sep_id >= 0;
    const uint8_t* s = (const uint8_t*)text;
    int64_t w = 0;
    for (int64_t i = 0; i < n_texts; ++i) {
        const int64_t a = offsets[i], b = offsets[i + 1];
        if (a < 0 || b < a || (b > a && !text)) return HR_E_INVALID;
        const int64_t w0 = w;
        if (special) {
            if (w >= ids_cap) return HR_E_INVALID;
            ids_out[w++] = cls_id;
        }
        int64_t n = 0;
        int64_t p = a;
        while (p < b && (cap < 0 || n < cap)) {
            const uint8_t c = s[p];
            if (c >= 0x80) return HR_E_INVALID;  // ASCII only (the caller routes other texts to Python)
            if (is_space(c)) {
                ++p;
                continue;
            }
            uint32_t crc = 0xFFFFFFFFu;
            if (is_word(c)) {
                while (p < b && is_word(s[p])) {
                    crc = kCrc.t[(crc ^ lower(s[p])) & 0xFFu] ^ (crc >> 8);
                    ++p;
                }
            } else {
                crc = kCrc.t[(crc ^ c) & 0xFFu] ^ (crc >> 8);
                ++p;
            }
            if (w >= ids_cap) return HR_E_INVALID;
            ids_out[w++] = first_id + (int64_t)((crc ^ 0xFFFFFFFFu) % (uint64_t)span);
            ++n;
        }
        for (int64_t q = p; q < b; ++q)  // (past the cap: the rest must still be ASCII)
            if (s[q] >= 0x80) return HR_E_INVALID;
        if (special) {
            if (w >= ids_cap) return HR_E_INVALID;
            ids_out[w++] = sep_id;
        }
        lengths_out[i] = w - w0;
    }
    return HR_OK;
}
