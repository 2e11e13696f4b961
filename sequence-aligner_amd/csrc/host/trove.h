// trove.h -- replay of GNU Trove 3.0.3 TIntObjectHashMap slot layout (host).
//
// The reference keeps KmerData, PairData and DispatchData in Trove maps
// (KmerTable.scala:26-37) and emits records in their iteration order, so a
// byte-identical .ovl needs the final slot of every key.  Semantics (read from
// lib/trove.jar's class files): initial capacity nextPrime(20)=23,
// load 0.5f, hash(int)=value, idx = (key & 0x7fffffff) % cap, collisions step
// idx -= 1 + h % (cap-2), growth to nextPrime(cap<<1) when size > maxSize
// (= min(cap-1, (int)(cap*0.5f))), rehash reinserting old slots high -> low,
// iteration from slot cap-1 down to 0.  Only insertions happen in this path.
#pragma once
#include <stdint.h>
#include <vector>

#include "trove_primes.h"

namespace sa {

class TroveLayout {
public:
    TroveLayout() { reset(); }

    void reset() {
        const float f = 10.0f / 0.5f;  // HashFunctions.fastCeil(initialCapacity / loadFactor)
        int32_t c = (int32_t)f;
        if (f - (float)c > 0.0f) ++c;
        alloc(next_prime(c));
        size_ = 0;
        compute_max_size();
    }

    // put(key, val) for a key not yet present; returns false if it was present
    // (the value is the caller's payload -- e.g. the key's index in its arrays --
    // and moves with the key through every rehash, so iteration needs no lookup)
    bool insert(int32_t key, int32_t val = 0) {
        int32_t slot;
        bool fresh = probe_insert(key, &slot);
        if (!fresh) return false;
        vals_[(size_t)slot] = val;
        if (consumed_free_) --free_;
        if (++size_ > max_size_ || free_ == 0) {
            rehash(size_ > max_size_ ? next_prime(cap_ << 1) : cap_);
            compute_max_size();
        }
        return true;
    }

    int32_t capacity() const { return cap_; }
    int32_t size() const { return size_; }

    // keys in THashPrimitiveIterator order (slot cap-1 .. 0)
    template <class F>
    void for_each(F f) const {
        for (int32_t i = cap_; i-- > 0;)
            if (full_[(size_t)i]) f(keys_[(size_t)i]);
    }
    // (key, value) in the same order
    template <class F>
    void for_each_kv(F f) const {
        for (int32_t i = cap_; i-- > 0;)
            if (full_[(size_t)i]) f(keys_[(size_t)i], vals_[(size_t)i]);
    }

    static int32_t next_prime(int32_t desired) {
        int lo = 0, hi = TROVE_NPRIMES - 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            if (trove_primes[mid] < desired) lo = mid + 1;
            else if (trove_primes[mid] > desired) hi = mid - 1;
            else return trove_primes[mid];
        }
        return trove_primes[lo];
    }

private:
    // Separate arrays: a probe reads the 1-byte occupancy array (6.6 MB at configs[0]'s
    // 6.58M-slot PairData table -- cache-resident) and touches the keys only on an
    // occupied slot; the values are written once and read by iteration / rehash.  (Key
    // and value in one 8-byte slot probed 1.7x slower on the 3.1M-key replay.)
    void alloc(int32_t cap) {
        cap_ = cap;
        keys_.assign((size_t)cap, 0);
        vals_.resize((size_t)cap);
        full_.assign((size_t)cap, 0);
    }
    void compute_max_size() {
        const int32_t lf = (int32_t)((float)cap_ * 0.5f);
        max_size_ = cap_ - 1 < lf ? cap_ - 1 : lf;
        free_ = cap_ - size_;
    }
    bool probe_insert(int32_t key, int32_t *slot) {
        const int32_t length = cap_;
        const int32_t hash = key & 0x7fffffff;
        int32_t index = hash % length;
        consumed_free_ = false;
        if (!full_[(size_t)index]) {
            consumed_free_ = true;
            keys_[(size_t)index] = key; full_[(size_t)index] = 1; *slot = index;
            return true;
        }
        if (keys_[(size_t)index] == key) { *slot = index; return false; }
        const int32_t probe = 1 + (hash % (length - 2));
        for (;;) {
            index -= probe;
            if (index < 0) index += length;
            if (!full_[(size_t)index]) {
                consumed_free_ = true;
                keys_[(size_t)index] = key; full_[(size_t)index] = 1; *slot = index;
                return true;
            }
            if (keys_[(size_t)index] == key) { *slot = index; return false; }
        }
    }
    void rehash(int32_t newcap) {
        std::vector<int32_t> ok, ov;
        std::vector<uint8_t> of;
        ok.swap(keys_);
        ov.swap(vals_);
        of.swap(full_);
        const int32_t oldcap = cap_;
        alloc(newcap);
        for (int32_t i = oldcap; i-- > 0;) {
            if (of[(size_t)i]) {
                int32_t s;
                probe_insert(ok[(size_t)i], &s);
                vals_[(size_t)s] = ov[(size_t)i];
            }
        }
    }

    std::vector<int32_t> keys_, vals_;
    std::vector<uint8_t> full_;
    int32_t cap_ = 0, size_ = 0, free_ = 0, max_size_ = 0;
    bool consumed_free_ = false;
};

}  // namespace sa
