// Deterministic synthetic tweet stream; see synth.h.
#include "../common/host_threads.h"
#include "synth.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace twtml {
namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

struct Rng {  // xoshiro256** seeded by splitmix64(seed, index)
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) { x = splitmix64(x); v = x; }
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  inline uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  inline double uniform() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  inline uint32_t below(uint32_t n) { return uint32_t((next() >> 32) * uint64_t(n) >> 32); }
  inline double normal() {  // Box-Muller
    double u1 = uniform(), u2 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

// ---------------------------------------------------------------- vocabulary
const char* kWords[] = {
    "the", "to", "and", "a", "of", "in", "is", "for", "on", "you", "it", "with", "that", "this",
    "be", "are", "at", "my", "we", "i", "so", "your", "all", "have", "me", "not", "just", "but",
    "from", "can", "will", "by", "what", "out", "new", "now", "up", "get", "one", "do", "more",
    "our", "day", "if", "about", "time", "like", "no", "how", "today", "people", "when", "love",
    "see", "they", "go", "who", "an", "good", "great", "know", "was", "has", "best", "don't",
    "it's", "year", "back", "need", "first", "here", "world", "life", "via", "happy", "there",
    "make", "think", "right", "want", "their", "been", "still", "night", "only", "never", "over",
    "really", "why", "would", "thank", "thanks", "us", "look", "he", "she", "her", "his", "them",
    "these", "video", "watch", "game", "win", "free", "live", "news", "breaking", "music",
    "follow", "check", "please", "help", "going", "week", "man", "god", "home", "tonight",
    "team", "season", "show", "big", "read", "last", "next", "vote", "night", "family", "friends",
    "fans", "photo", "story", "morning", "weekend", "birthday", "amazing", "beautiful", "proud",
    "congratulations", "support", "share", "retweet", "giveaway", "chance", "enter", "official",
    "announce", "album", "tour", "tickets", "trailer", "episode", "stream", "update", "report",
    "president", "election", "government", "police", "city", "school", "water", "climate",
    "health", "covid", "vaccine", "data", "science", "tech", "apple", "google", "crypto",
    "bitcoin", "market", "price", "money", "business", "job", "work", "career", "learn", "code",
    "ai", "model", "football", "soccer", "goal", "match", "player", "coach", "league", "cup",
    "final", "champions", "nba", "nfl", "movie", "film", "star", "actor", "song", "dance", "art",
    "food", "coffee", "pizza", "travel", "beach", "summer", "winter", "rain", "sun", "moon",
    "dog", "cat", "baby", "kids", "mom", "dad", "sister", "brother", "wife", "husband", "girl",
    "boy", "everyone", "someone", "nothing", "everything", "always", "forever", "again", "ever",
    "never", "tomorrow", "yesterday", "soon", "finally", "literally", "actually", "seriously",
    "omg", "lol", "lmao", "wow", "yes", "yeah", "okay", "ok", "pls", "thx", "via", "rt", "amp",
    "must", "should", "could", "may", "might", "did", "does", "doing", "done", "said", "says",
    "says", "made", "makes", "take", "took", "give", "gave", "find", "found", "call", "called",
    "2024", "2025", "100", "1st", "24/7", "10k", "5", "#1", "&", "-", "...", ":", "!", "?", "!!",
};
constexpr int kNumWords = sizeof(kWords) / sizeof(kWords[0]);

struct Keyword { const char* w; double score; };
const Keyword kKeywords[] = {
    {"breaking", 180}, {"giveaway", 260}, {"win", 110}, {"free", 90}, {"official", 140},
    {"announce", 150}, {"album", 120}, {"tour", 100}, {"tickets", 95}, {"trailer", 130},
    {"retweet", 170}, {"vote", 80}, {"election", 70}, {"president", 60}, {"champions", 90},
    {"final", 70}, {"goal", 60}, {"congratulations", 75}, {"birthday", 55}, {"love", 30},
    {"lol", -20}, {"me", -15}, {"i", -10}, {"my", -12},
};

// Non-Latin / accented words (UTF-8) and emoji code points for "unicode" tweets.
const char* kIntlWords[] = {
    "café", "niño", "über", "straße", "façade", "élève", "ação", "smörgåsbord", "привет", "мир",
    "спасибо", "γεια", "σας", "καλημέρα", "こんにちは", "ありがとう", "你好", "世界", "谢谢",
    "안녕하세요", "مرحبا", "شكرا", "שלום", "नमस्ते", "ধন্যবাদ", "สวัสดี", "Ünïcödé", "ÇA", "ŞEHİR",
    "ΑΘΗΝΑ", "МОСКВА", "Ärger", "ÉTÉ",
};
constexpr int kNumIntl = sizeof(kIntlWords) / sizeof(kIntlWords[0]);
const char* kSpecialWords[] = {"İstanbul", "İZMİR", "ΟΔΟΣ", "ΣΟΦΙΑ", "ΛΟΓΟΣ.", "ΣΑΣ", "𐐀𐐁𐐂",
                               "𞤀𞤁", "ΜΑΣ ΤΟΥΣ"};
constexpr int kNumSpecial = sizeof(kSpecialWords) / sizeof(kSpecialWords[0]);
const uint32_t kEmoji[] = {0x1F600, 0x1F602, 0x1F525, 0x2764,  0x1F44D, 0x1F64F, 0x1F389,
                           0x1F62D, 0x1F60D, 0x2728,  0x1F4AF, 0x1F680, 0x1F3C6, 0x26BD,
                           0x1F3B6, 0x1F1FA, 0x1F1F8, 0x1F914};
constexpr int kNumEmoji = sizeof(kEmoji) / sizeof(kEmoji[0]);

void utf8_to_utf16(const char* s, std::vector<uint16_t>& out) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
  while (*p) {
    uint32_t cp;
    if (*p < 0x80) { cp = *p++; }
    else if ((*p >> 5) == 6) { cp = (uint32_t(p[0] & 0x1F) << 6) | (p[1] & 0x3F); p += 2; }
    else if ((*p >> 4) == 14) {
      cp = (uint32_t(p[0] & 0x0F) << 12) | (uint32_t(p[1] & 0x3F) << 6) | (p[2] & 0x3F); p += 3;
    } else {
      cp = (uint32_t(p[0] & 0x07) << 18) | (uint32_t(p[1] & 0x3F) << 12) |
           (uint32_t(p[2] & 0x3F) << 6) | (p[3] & 0x3F);
      p += 4;
    }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back(uint16_t(0xD800 + (cp >> 10)));
      out.push_back(uint16_t(0xDC00 + (cp & 0x3FF)));
    } else {
      out.push_back(uint16_t(cp));
    }
  }
}

struct Vocab {
  std::vector<std::vector<uint16_t>> words, intl, special, emoji;
  std::vector<double> score;     // keyword score per word
  std::vector<double> cdf;       // Zipf-like sampling CDF over words
  Vocab() {
    for (int i = 0; i < kNumWords; ++i) {
      words.emplace_back();
      utf8_to_utf16(kWords[i], words.back());
      double sc = 0;
      for (const auto& k : kKeywords)
        if (std::strcmp(k.w, kWords[i]) == 0) sc = k.score;
      score.push_back(sc);
    }
    for (int i = 0; i < kNumIntl; ++i) { intl.emplace_back(); utf8_to_utf16(kIntlWords[i], intl.back()); }
    for (int i = 0; i < kNumSpecial; ++i) {
      special.emplace_back();
      utf8_to_utf16(kSpecialWords[i], special.back());
    }
    for (int i = 0; i < kNumEmoji; ++i) {
      emoji.emplace_back();
      uint32_t cp = kEmoji[i];
      if (cp >= 0x10000) {
        cp -= 0x10000;
        emoji.back().push_back(uint16_t(0xD800 + (cp >> 10)));
        emoji.back().push_back(uint16_t(0xDC00 + (cp & 0x3FF)));
      } else {
        emoji.back().push_back(uint16_t(cp));
      }
    }
    double acc = 0;
    for (int i = 0; i < kNumWords; ++i) { acc += 1.0 / (i + 3.0); cdf.push_back(acc); }
    for (auto& c : cdf) c /= acc;
  }
  int sample_word(Rng& r) const {
    const double u = r.uniform();
    return int(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()) % kNumWords;
  }
};

const Vocab& vocab() {
  static const Vocab v;
  return v;
}

// ------------------------------------------------- realistic vocabulary (vocab=1)
// Words are generated once per vocab_size from a fixed seed (every rank and
// thread sees the same language), per script, each list sampled Zipf-style.
enum Script { kLatin, kAccent, kCyr, kGreek, kCjk, kKana, kHangul, kArabic, kDeva, kThai, kHebrew, kNumScripts };
// share of the vocabulary, and of the unicode tweets, per script
const double kScriptShare[kNumScripts] = {0.50, 0.07, 0.10, 0.03, 0.14, 0.04, 0.04, 0.03, 0.02, 0.015, 0.015};
const double kScriptTweets[kNumScripts] = {0.0, 0.22, 0.18, 0.06, 0.18, 0.10, 0.08, 0.08, 0.04, 0.03, 0.03};

struct ZipfList {
  std::vector<std::vector<uint16_t>> w;
  std::vector<double> cdf;
  void finish(double s) {
    double acc = 0;
    cdf.clear();
    for (size_t i = 0; i < w.size(); ++i) { acc += 1.0 / std::pow(double(i) + 2.0, s); cdf.push_back(acc); }
    for (auto& c : cdf) c /= acc;
  }
  const std::vector<uint16_t>& sample(Rng& r) const {
    const size_t i = size_t(std::lower_bound(cdf.begin(), cdf.end(), r.uniform()) - cdf.begin());
    return w[std::min(i, w.size() - 1)];
  }
  size_t sample_index(Rng& r) const {
    return std::min(size_t(std::lower_bound(cdf.begin(), cdf.end(), r.uniform()) - cdf.begin()), w.size() - 1);
  }
};

struct WideVocab {
  ZipfList list[kNumScripts];
  std::vector<double> latin_score;   // label effect of Latin words (keywords)
  double tweet_cdf[kNumScripts];

  explicit WideVocab(int size) {
    Rng r(0xC0FFEE1234ULL ^ uint64_t(size));
    static const char* on[] = {"", "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t",
                               "v", "w", "y", "z", "bl", "br", "ch", "cl", "cr", "dr", "fl", "fr", "gl", "gr",
                               "pl", "pr", "sh", "sl", "sp", "st", "str", "th", "tr", "wh", "qu", "sk", "sn"};
    static const char* nu[] = {"a", "e", "i", "o", "u", "a", "e", "i", "o", "ai", "ea", "ee", "ie", "oo", "ou", "y"};
    static const char* co[] = {"", "", "", "n", "r", "s", "t", "l", "m", "ng", "nd", "st", "rt", "ck", "x", "ll"};
    auto latin_word = [&](std::vector<uint16_t>& w) {
      const double u = r.uniform();
      const int syl = u < 0.3 ? 1 : u < 0.7 ? 2 : u < 0.9 ? 3 : 4;
      for (int k = 0; k < syl; ++k) {
        for (const char* c = on[r.below(sizeof(on) / sizeof(on[0]))]; *c; ++c) w.push_back(uint16_t(*c));
        for (const char* c = nu[r.below(sizeof(nu) / sizeof(nu[0]))]; *c; ++c) w.push_back(uint16_t(*c));
        for (const char* c = co[r.below(sizeof(co) / sizeof(co[0]))]; *c; ++c) w.push_back(uint16_t(*c));
      }
    };
    // Latin-1 vowels with accents, by base vowel (a e i o u) + n, c, s
    static const uint16_t acc_a[] = {0xE0, 0xE1, 0xE2, 0xE4, 0xE3, 0xE5};
    static const uint16_t acc_e[] = {0xE8, 0xE9, 0xEA, 0xEB};
    static const uint16_t acc_i[] = {0xEC, 0xED, 0xEE, 0xEF};
    static const uint16_t acc_o[] = {0xF2, 0xF3, 0xF4, 0xF6, 0xF5, 0xF8};
    static const uint16_t acc_u[] = {0xF9, 0xFA, 0xFB, 0xFC};
    auto range_word = [&](std::vector<uint16_t>& w, uint16_t lo, uint16_t n, int lmin, int lmax,
                          const std::vector<uint16_t>* skip = nullptr) {
      const int L = lmin + int(r.below(uint32_t(lmax - lmin + 1)));
      for (int k = 0; k < L; ++k) {
        uint16_t c;
        do { c = uint16_t(lo + r.below(n)); } while (skip && std::find(skip->begin(), skip->end(), c) != skip->end());
        w.push_back(c);
      }
    };
    // CJK / Hangul characters are themselves Zipf distributed (common ones common)
    ZipfList cjk_chars, hangul_chars;
    for (int i = 0; i < 6000; ++i) cjk_chars.w.push_back({uint16_t(0x4E00 + (i * 2654435761u) % 20902u)});
    cjk_chars.finish(0.9);
    for (int i = 0; i < 2400; ++i) hangul_chars.w.push_back({uint16_t(0xAC00 + (i * 40503u) % 11172u)});
    hangul_chars.finish(0.9);
    const std::vector<uint16_t> greek_skip = {0x3C2};   // final sigma only comes from lowering
    for (int s = 0; s < kNumScripts; ++s) {
      const int n = std::max(16, int(double(size) * kScriptShare[s]));
      auto& L = list[s].w;
      L.reserve(size_t(n));
      while (int(L.size()) < n) {
        std::vector<uint16_t> w;
        switch (s) {
          case kLatin: latin_word(w); break;
          case kAccent: {
            latin_word(w);
            bool any = false;
            for (auto& c : w) {
              if (r.uniform() > 0.35) continue;
              switch (c) {
                case 'a': c = acc_a[r.below(6)]; any = true; break;
                case 'e': c = acc_e[r.below(4)]; any = true; break;
                case 'i': c = acc_i[r.below(4)]; any = true; break;
                case 'o': c = acc_o[r.below(6)]; any = true; break;
                case 'u': c = acc_u[r.below(4)]; any = true; break;
                case 'n': c = 0xF1; any = true; break;
                case 'c': c = 0xE7; any = true; break;
                case 's': if (r.uniform() < 0.3) { c = 0xDF; any = true; } break;
                default: break;
              }
            }
            if (!any) w.push_back(0xE9);
            break;
          }
          case kCyr: range_word(w, 0x430, 32, 2, 10); if (r.uniform() < 0.05) w.push_back(0x451); break;
          case kGreek: range_word(w, 0x3B1, 25, 2, 9, &greek_skip); break;
          case kCjk: {
            const int len = 1 + int(r.below(4));
            for (int k = 0; k < len; ++k) w.push_back(cjk_chars.sample(r)[0]);
            break;
          }
          case kKana: range_word(w, r.uniform() < 0.5 ? 0x3041 : 0x30A1, 86, 2, 6); break;
          case kHangul: {
            const int len = 1 + int(r.below(4));
            for (int k = 0; k < len; ++k) w.push_back(hangul_chars.sample(r)[0]);
            break;
          }
          case kArabic: range_word(w, 0x621, 42, 2, 8); break;
          case kDeva: range_word(w, 0x905, 53, 2, 8); break;
          case kThai: range_word(w, 0xE01, 46, 2, 8); break;
          default: range_word(w, 0x5D0, 27, 2, 7); break;
        }
        L.push_back(std::move(w));
      }
      list[s].finish(1.0);
    }
    latin_score.assign(list[kLatin].w.size(), 0.0);
    for (auto& sc : latin_score)
      if (r.uniform() < 0.03) sc = 60.0 * r.normal();
    double acc = 0;
    for (int s = 0; s < kNumScripts; ++s) { acc += kScriptTweets[s]; tweet_cdf[s] = acc; }
    for (auto& c : tweet_cdf) c /= acc;
  }
};

const WideVocab& wide_vocab(int size) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<WideVocab>> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto& v = cache[size];
  if (!v) v.reset(new WideVocab(size));
  return *v;
}

// upper-case of a lower-case letter of the generated scripts (0 if none)
inline uint16_t upper_of(uint16_t c) {
  if (c >= 'a' && c <= 'z') return uint16_t(c - 32);
  if (c >= 0xE0 && c <= 0xFE && c != 0xF7) return uint16_t(c - 32);
  if (c >= 0x430 && c <= 0x44F) return uint16_t(c - 32);
  if (c >= 0x3B1 && c <= 0x3C9 && c != 0x3C2) return uint16_t(c - 32);
  return 0;
}

struct RowOut {
  int64_t rt, fol, fav, fri, cre;
  uint8_t is_rt;
};

void gen_row_wide(const SynthParams& p, uint64_t idx, std::vector<uint16_t>& text, RowOut& o) {
  const WideVocab& V = wide_vocab(p.vocab_size);
  const Vocab& T = vocab();
  Rng r(splitmix64(p.seed * 0x9E3779B97F4A7C15ULL + 0x5851F42D4C957F2DULL) ^ splitmix64(idx));
  o.is_rt = r.uniform() < p.retweet_fraction ? 1 : 0;
  o.fol = int64_t(std::floor(std::pow(10.0, r.uniform() * 7.0)));
  o.fav = int64_t(std::floor(std::pow(10.0, r.uniform() * 5.5)));
  o.fri = int64_t(std::floor(std::pow(10.0, r.uniform() * 3.7)));
  o.cre = p.now_ms - int64_t(r.uniform() * double(p.max_age_ms));
  const int32_t lo = std::max<int32_t>(1, p.min_len);
  const int32_t hi = std::max<int32_t>(lo, p.max_len);
  const size_t L = size_t(lo + int32_t(r.below(uint32_t(hi - lo + 1))));
  int script = kLatin;
  if (r.uniform() < p.unicode_fraction) {
    const double u = r.uniform();
    script = int(std::lower_bound(V.tweet_cdf, V.tweet_cdf + kNumScripts, u) - V.tweet_cdf);
    if (script >= kNumScripts) script = kNumScripts - 1;
  }
  bool special = r.uniform() < p.special_fraction;
  bool url_done = false;
  const bool shout = r.uniform() < 0.01;   // ALL CAPS tweet
  double kw = 0;
  const size_t start = text.size();
  std::vector<uint16_t> tmp;
  // CJK, kana and Thai text runs words together (no spaces between them)
  const bool nospace = script == kCjk || script == kKana || script == kThai;
  bool prev_script = false;
  while (text.size() - start < L) {
    const double u = r.uniform();
    const std::vector<uint16_t>* w = nullptr;
    const bool glue = nospace && prev_script && u >= 0.12 && u <= 0.985;
    if (text.size() > start && !glue) text.push_back(' ');
    prev_script = false;
    if (special) {
      w = &T.special[r.below(T.special.size())];
      special = false;
    } else if (!url_done && u > 0.985) {
      static const char* kUrl = "https://t.co/";
      for (const char* c = kUrl; *c; ++c) text.push_back(uint16_t(*c));
      for (int k = 0; k < 10; ++k) {
        const uint32_t d = r.below(62);
        text.push_back(uint16_t(d < 10 ? '0' + d : d < 36 ? 'a' + d - 10 : 'A' + d - 36));
      }
      url_done = true;
      continue;
    } else if (u < (script == kLatin ? 0.01 : 0.08)) {
      w = &T.emoji[r.below(T.emoji.size())];
    } else if (u < 0.12) {   // @handle: fresh random name
      text.push_back('@');
      const int hl = 4 + int(r.below(11));
      for (int k = 0; k < hl; ++k) {
        const uint32_t d = r.below(37);
        text.push_back(uint16_t(d < 10 ? '0' + d : d < 36 ? 'a' + d - 10 : '_'));
      }
      continue;
    } else {
      int s = script;
      if (script == kLatin) s = r.uniform() < 0.05 ? kAccent : kLatin;
      else if (r.uniform() < 0.35) s = kLatin;
      const size_t wi = V.list[s].sample_index(r);
      w = &V.list[s].w[wi];
      prev_script = s == script;
      if (s == kLatin) kw += V.latin_score[wi];
      if (u < 0.17) text.push_back('#');
    }
    const double cas = r.uniform();
    tmp.assign(w->begin(), w->end());
    for (size_t k = 0; k < tmp.size(); ++k) {
      const uint16_t up = upper_of(tmp[k]);
      if (up && (shout || cas < 0.015 || (cas < 0.13 && k == 0))) tmp[k] = up;
    }
    text.insert(text.end(), tmp.begin(), tmp.end());
    const double pu = r.uniform();
    if (pu < 0.06) text.push_back(pu < 0.02 ? ',' : pu < 0.04 ? '.' : '!');
  }
  size_t len = std::min(text.size() - start, L);
  if (len > 0) {
    const uint16_t last = text[start + len - 1];
    if (last >= 0xD800 && last <= 0xDBFF) --len;
  }
  if (len == 0) { text.resize(start); text.push_back('x'); len = 1; }
  text.resize(start + len);
  double label = p.rt_base + p.rt_slope * std::log10(1.0 + double(o.fol)) + kw + p.rt_noise * r.normal();
  if (r.uniform() < p.rt_tail) label = std::pow(10.0, r.uniform() * std::log10(double(std::max<int64_t>(2, p.rt_hi))));
  label = std::min(double(p.rt_hi), std::max(double(p.rt_lo), std::round(label)));
  o.rt = int64_t(label);
}

void gen_row(const SynthParams& p, uint64_t idx, std::vector<uint16_t>& text, RowOut& o) {
  const Vocab& V = vocab();
  Rng r(splitmix64(p.seed * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL) ^ splitmix64(idx));
  o.is_rt = r.uniform() < p.retweet_fraction ? 1 : 0;
  o.fol = int64_t(std::floor(std::pow(10.0, r.uniform() * 7.0)));
  o.fav = int64_t(std::floor(std::pow(10.0, r.uniform() * 5.5)));
  o.fri = int64_t(std::floor(std::pow(10.0, r.uniform() * 3.7)));
  o.cre = p.now_ms - int64_t(r.uniform() * double(p.max_age_ms));
  const int32_t lo = std::max<int32_t>(1, p.min_len);
  const int32_t hi = std::max<int32_t>(lo, p.max_len);
  const size_t L = size_t(lo + int32_t(r.below(uint32_t(hi - lo + 1))));
  const bool intl = r.uniform() < p.unicode_fraction;
  bool special = r.uniform() < p.special_fraction;
  bool url_done = false;
  double kw = 0;
  const size_t start = text.size();
  while (text.size() - start < L) {
    if (text.size() > start) text.push_back(' ');
    const double u = r.uniform();
    const std::vector<uint16_t>* w;
    int wi = -1;
    if (special) {
      w = &V.special[r.below(V.special.size())];
      special = false;
    } else if (intl && u < 0.12) {
      w = &V.emoji[r.below(V.emoji.size())];
    } else if (intl && u < 0.30) {
      w = &V.intl[r.below(V.intl.size())];
    } else if (!url_done && u > 0.985) {
      static const char* kUrl = "https://t.co/";
      for (const char* c = kUrl; *c; ++c) text.push_back(uint16_t(*c));
      for (int k = 0; k < 10; ++k) {
        const uint32_t d = r.below(62);
        text.push_back(uint16_t(d < 10 ? '0' + d : d < 36 ? 'a' + d - 10 : 'A' + d - 36));
      }
      url_done = true;
      continue;
    } else {
      wi = V.sample_word(r);
      w = &V.words[wi];
      kw += V.score[wi];
      if (u < 0.05) text.push_back('#');
      else if (u < 0.09) text.push_back('@');
    }
    const double cas = r.uniform();
    for (size_t k = 0; k < w->size(); ++k) {
      uint16_t c = (*w)[k];
      if (c >= 'a' && c <= 'z' && (cas < 0.015 || (cas < 0.13 && k == 0))) c = uint16_t(c - 32);
      text.push_back(c);
    }
  }
  // truncate to L units without splitting a surrogate pair
  size_t len = std::min(text.size() - start, L);
  if (len > 0) {
    const uint16_t last = text[start + len - 1];
    if (last >= 0xD800 && last <= 0xDBFF) --len;
  }
  if (len == 0) { text.resize(start); text.push_back('x'); len = 1; }
  text.resize(start + len);
  double label = p.rt_base + p.rt_slope * std::log10(1.0 + double(o.fol)) + kw + p.rt_noise * r.normal();
  if (r.uniform() < p.rt_tail) label = std::pow(10.0, r.uniform() * std::log10(double(std::max<int64_t>(2, p.rt_hi))));
  label = std::min(double(p.rt_hi), std::max(double(p.rt_lo), std::round(label)));
  o.rt = int64_t(label);
}

}  // namespace

size_t synth_max_units(const SynthParams& p, size_t n) {
  return n * size_t(std::max<int32_t>(1, p.max_len) + 1);
}

int64_t synth_generate(const SynthParams& p, uint64_t start, size_t n, uint16_t* text,
                       size_t text_cap, int64_t* offsets, uint8_t* is_rt, int64_t* scalars,
                       int nthreads) {
  (void)vocab();  // initialise statics before threads start
  if (p.vocab == 1) (void)wide_vocab(p.vocab_size);
  if (n == 0) { offsets[0] = 0; return 0; }
  int T = nthreads > 0 ? nthreads : host_threads();
  T = std::max(1, std::min<int>(T, int((n + 4095) / 4096)));
  std::vector<std::vector<uint16_t>> bufs(T);
  std::vector<size_t> row0(T + 1);
  for (int t = 0; t <= T; ++t) row0[t] = n * size_t(t) / size_t(T);
  auto work = [&](int t) {
    auto& buf = bufs[t];
    buf.reserve((row0[t + 1] - row0[t]) * size_t(p.max_len / 2 + 8));
    RowOut o;
    for (size_t i = row0[t]; i < row0[t + 1]; ++i) {
      if (p.vocab == 1) gen_row_wide(p, start + i, buf, o);
      else gen_row(p, start + i, buf, o);
      offsets[i + 1] = int64_t(buf.size());  // local end; fixed up below
      is_rt[i] = o.is_rt;
      scalars[0 * n + i] = o.rt;
      scalars[1 * n + i] = o.fol;
      scalars[2 * n + i] = o.fav;
      scalars[3 * n + i] = o.fri;
      scalars[4 * n + i] = o.cre;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  size_t total = 0;
  std::vector<size_t> base(T);
  for (int t = 0; t < T; ++t) { base[t] = total; total += bufs[t].size(); }
  if (total > text_cap) return -int64_t(total);
  auto fix = [&](int t) {
    std::memcpy(text + base[t], bufs[t].data(), bufs[t].size() * sizeof(uint16_t));
    for (size_t i = row0[t]; i < row0[t + 1]; ++i) offsets[i + 1] += int64_t(base[t]);
  };
  th.clear();
  for (int t = 1; t < T; ++t) th.emplace_back(fix, t);
  fix(0);
  for (auto& x : th) x.join();
  offsets[0] = 0;
  return int64_t(total);
}

}  // namespace twtml
