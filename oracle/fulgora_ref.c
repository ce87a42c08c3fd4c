/*
 * fulgora_ref.c — CPU ORACLE for the Titan OLAP path (test infrastructure; see header).
 *
 * Every function cites the reference file:line it restates.  Paths are relative to
 * /root/reference/titan-core/src/main/java/com/thinkaurelius/titan/ unless noted;
 * "tmain/" = titan-test/src/main/java/com/thinkaurelius/titan/.
 */
#define _GNU_SOURCE
#include "fulgora_ref.h"
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>

/* ===================================================================== buffers */
static void buf_put(fr_buf* b, uint8_t x) {
    if (b->len == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 64;
        b->p = (uint8_t*)realloc(b->p, b->cap);
    }
    b->p[b->len++] = x;
}
void fr_buf_free(fr_buf* b) { free(b->p); b->p = NULL; b->len = b->cap = 0; }

/* ===================================================================== VariableLong */
/* graphdb/database/idhandling/VariableLong.java */
static int bit_length(uint64_t v) {            /* unsignedBitLength :71-73 */
    return v == 0 ? 1 : 64 - __builtin_clzll(v);
}
static int num_blocks(int bits) { return (bits - 1) / 7 + 1; }   /* :66-69 */

static void write_unsigned_n(fr_buf* b, int offset, uint64_t value) {   /* :46-57 */
    while (offset > 0) {
        offset -= 7;
        uint8_t x = (uint8_t)((value >> offset) & 0x7F);
        if (offset == 0) x |= 0x80;             /* STOP_MASK on the last byte */
        buf_put(b, x);
    }
}
static uint64_t read_unsigned(const uint8_t* d, size_t* pos) {          /* :30-38 */
    uint64_t value = 0;
    int8_t x;
    do {
        x = (int8_t)d[(*pos)++];
        value = (value << 7) | (uint64_t)(x & 0x7F);
    } while (x >= 0);
    return value;
}
int fr_vl_positive_length(int64_t v) { return num_blocks(bit_length((uint64_t)v)); }
void fr_vl_write_positive(fr_buf* b, int64_t v) {                       /* :84-87 */
    write_unsigned_n(b, num_blocks(bit_length((uint64_t)v)) * 7, (uint64_t)v);
}
int64_t fr_vl_read_positive(const uint8_t* d, size_t* pos) { return (int64_t)read_unsigned(d, pos); }

static uint64_t to_unsigned(int64_t v) {                                 /* convert2Unsigned :112-115 */
    uint64_t a = v < 0 ? (uint64_t)(-(v)) : (uint64_t)v;
    return (a << 1) | (v < 0 ? 1u : 0u);
}
static int64_t from_unsigned(uint64_t u) {                               /* :117-119 */
    return (u & 1) ? -(int64_t)(u >> 1) : (int64_t)(u >> 1);
}
void fr_vl_write(fr_buf* b, int64_t v) {                                 /* :125-127 */
    uint64_t u = to_unsigned(v);
    write_unsigned_n(b, num_blocks(bit_length(u)) * 7, u);
}
int64_t fr_vl_read(const uint8_t* d, size_t* pos) { return from_unsigned(read_unsigned(d, pos)); }

void fr_vl_write_positive_with_prefix(fr_buf* b, int64_t value, int64_t prefix, int prefix_len) {
    /* :139-164 */
    int delta_len = 8 - prefix_len;
    uint8_t first = (uint8_t)(prefix << delta_len);
    uint64_t v = (uint64_t)value;
    int value_len = bit_length(v);
    int mod = value_len % 7;
    if (mod <= delta_len - 1) {
        int offset = value_len - mod;
        first |= (uint8_t)(v >> offset);
        v = offset >= 64 ? v : (v & ((1ULL << offset) - 1));
        value_len -= mod;
    } else {
        value_len += 7 - mod;
    }
    if (value_len > 0) first |= (uint8_t)(1 << (delta_len - 1));   /* continue mask */
    buf_put(b, first);
    if (value_len > 0) write_unsigned_n(b, value_len, v);
}
void fr_vl_read_positive_with_prefix(const uint8_t* d, size_t* pos, int prefix_len,
                                     int64_t* value, int64_t* prefix) {  /* :171-186 */
    int first = d[(*pos)++];
    int delta_len = 8 - prefix_len;
    *prefix = first >> delta_len;
    uint64_t v = (uint64_t)(first & ((1 << (delta_len - 1)) - 1));
    if ((first >> (delta_len - 1)) & 1) {
        size_t p0 = *pos;
        uint64_t rem = read_unsigned(d, pos);
        size_t dp = *pos - p0;
        v = (v << (dp * 7)) + rem;
    }
    *value = (int64_t)v;
}
int fr_vl_backward_length(int64_t value) {                               /* :247-252 */
    int bl = bit_length((uint64_t)value);
    int nb = 1 + (bl <= 4 ? 0 : (1 + (bl - 5) / 7));
    return nb < 3 ? 3 : nb;
}
void fr_vl_write_positive_backward(fr_buf* b, int64_t value) {          /* :234-245 */
    int nbytes = fr_vl_backward_length(value);
    int prefix_len = nbytes - 3;
    uint8_t x = (uint8_t)((prefix_len << 4) | 0x80);
    for (int i = nbytes - 1; i >= 0; i--) {
        x |= (uint8_t)(0x7F & ((uint64_t)value >> (i * 7)));
        buf_put(b, x);
        x = 0;
    }
}
int64_t fr_vl_read_positive_backward(const uint8_t* d, size_t* pos) {   /* :254-272 */
    size_t position = *pos;
    int nbytes = 0;
    uint64_t value = 0;
    for (;;) {
        position--;
        int8_t x = (int8_t)d[position];
        if (x < 0) {
            value |= (uint64_t)(x & 0x0F) << (7 * nbytes);
            break;
        }
        value |= (uint64_t)x << (7 * nbytes);
        nbytes++;
    }
    *pos = position;
    return (int64_t)value;
}

/* ===================================================================== IDManager */
/* graphdb/idmanagement/IDManager.java: VertexIDType offsets/suffixes :45-345 */
int64_t fr_schema_id(int type, int64_t count) {                          /* getSchemaId :620-623 */
    static const int64_t suffix[4] = {5, 37, 21, 53};  /* User/System PropertyKey, User/System EdgeLabel */
    return (count << 6) | suffix[type];
}
int64_t fr_vertex_id(int64_t count, int64_t partition, int pb) {         /* constructId :428-437 */
    int64_t id = (count << pb) + partition;
    return (id << 3) | 0;                                                /* NormalVertex 000b */
}
int64_t fr_key_of(int64_t vid, int pb) {                                 /* getKey :461-473 */
    if ((vid & 3) == 1) return vid;                                      /* Schema 01b */
    int64_t partition = (int64_t)(((uint64_t)vid >> 3) & ((1ULL << pb) - 1));
    int64_t count = (int64_t)((uint64_t)vid >> (pb + 3));
    int64_t suffix = vid & 7;
    uint64_t high = pb == 0 ? 0 : ((uint64_t)partition << (64 - pb));
    return (int64_t)(high | ((uint64_t)count << 3) | (uint64_t)suffix);
}
int64_t fr_key_id(int64_t key, int pb) {                                 /* getKeyID :476-486 */
    if ((key & 3) == 1) return key;                                      /* Schema */
    int64_t suffix = key & 7;
    int poff = 64 - pb;
    int64_t partition = poff < 64 ? (int64_t)((uint64_t)key >> poff) : 0;
    int64_t count = (int64_t)(((uint64_t)key >> 3) & ((1ULL << (poff - 3)) - 1));
    int64_t id = (count << pb) + partition;
    return (id << 3) | suffix;
}
int fr_is_invisible(int64_t vid) { return (vid & 1) == 1; }              /* VertexIDType.Invisible 1b */
/* Vertex cuts ("partitioned" vertices, VertexIDType.PartitionedVertex suffix 010b :78-90). */
static int64_t partition_hash(int64_t id, int pb) {                      /* getPartitionHashForId :512-523 */
    uint64_t r = 0;
    for (int off = 0; off < 64; off += pb) r ^= ((uint64_t)id >> off) & ((1ULL << pb) - 1);
    return (int64_t)r;
}
int64_t fr_partitioned_vertex_id(int64_t count, int64_t partition, int pb) {   /* constructId :432-441 */
    return (((count << pb) + partition) << 3) | 2;
}
int fr_is_partitioned(int64_t vid, int pb) {                             /* isPartitionedVertex :557-559 */
    return (vid & 7) == 2 && ((uint64_t)vid >> (pb + 3)) > 0;            /* + isUserVertexId :454-457 */
}
int64_t fr_canonical_vertex_id(int64_t vid, int pb) {                    /* getCanonicalVertexId :530-534 */
    if (pb <= 0) return vid;                     /* no partition bits: one representative only */
    int64_t count = (int64_t)((uint64_t)vid >> (pb + 3));
    return fr_partitioned_vertex_id(count, partition_hash(count, pb), pb);   /* :525-528 */
}

/* ===================================================================== IDHandler */
/* graphdb/database/idhandling/IDHandler.java */
void fr_write_relation_type(fr_buf* b, int64_t type_id, int is_edge, int dir, int invisible) {
    /* writeRelationType :88-94; getPrefix :61-64 */
    int system = ((type_id & 63) == 37) || ((type_id & 63) == 53);
    int64_t stripped = ((int64_t)((uint64_t)type_id >> 6) << 1) + dir;
    int64_t prefix = ((system ? 0 : invisible ? 2 : 1) << 1) + (is_edge ? 1 : 0);
    fr_vl_write_positive_with_prefix(b, stripped, prefix, 3);
}
int fr_read_relation_type(const uint8_t* d, size_t* pos, int64_t* type_id, int* is_edge, int* dir) {
    /* readRelationType :116-127 */
    int64_t value, prefix;
    fr_vl_read_positive_with_prefix(d, pos, 3, &value, &prefix);
    int rel = (int)(prefix & 1), dr = (int)(value & 1);
    if (rel == 0 && dr == 1) return FR_E_CODEC;                          /* DirectionID.forId(1) */
    int system = (prefix >> 1) == 0;
    int64_t cnt = (int64_t)((uint64_t)value >> 1);
    if (cnt <= 0) return FR_E_CODEC;
    *type_id = fr_schema_id(rel ? (system ? 3 : 2) : (system ? 1 : 0), cnt);
    *is_edge = rel;
    *dir = dr;
    return FR_OK;
}

/* ===================================================================== Serializer */
static const fr_edge_type* find_type(const fr_schema* s, int64_t id) {
    for (int i = 0; i < s->n_edge_types; i++) if (s->edge_types[i].type_id == id) return &s->edge_types[i];
    return NULL;
}
static int key_datatype(const fr_schema* s, int64_t id) {
    for (int i = 0; i < s->n_property_keys; i++) if (s->property_keys[i].key_id == id) return s->property_keys[i].datatype;
    return 0;
}
static int is_unique(int mult, int dir) {                                /* Multiplicity.isUnique :59-70 */
    if (dir == 1) return mult == FR_ONE2MANY || mult == FR_ONE2ONE;
    return mult == FR_MANY2ONE || mult == FR_ONE2ONE;
}
static void put_be(fr_buf* b, uint64_t v, int n) { for (int i = n - 1; i >= 0; i--) buf_put(b, (uint8_t)(v >> (8 * i))); }
/* fr_prop's String convention (fulgora_ref.h). */
int fr_string_of(int64_t value, uint16_t* chars) {
    int n = 0;
    if (value == 0) return 0;
    if (value < 0) { chars[n++] = 0x00E9; chars[n++] = 0x2135; }
    uint64_t a = value < 0 ? (uint64_t)0 - (uint64_t)value : (uint64_t)value;
    char digits[24]; int nd = 0;
    while (a) { digits[nd++] = (char)('0' + a % 10); a /= 10; }
    while (nd) chars[n++] = (uint16_t)digits[--nd];
    return n;
}
static uint32_t float_bits(int64_t v) { float f = (float)v; uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t double_bits(int64_t v) { double f = (double)v; uint64_t u; memcpy(&u, &f, 8); return u; }
/* StringSerializer.write :142-186 (no compression below 16000 chars; ASCII or full UTF). */
static void write_string(fr_buf* b, int64_t value) {
    uint16_t c[32]; int n = fr_string_of(value, c), ascii = 1;
    for (int i = 0; i < n; i++) ascii &= c[i] <= 127;
    if (ascii) {
        fr_vl_write_positive(b, (n == 0 ? 1 : 2) << 4);          /* NO_COMPRESSION_OFFSET = 4 */
        for (int i = 0; i < n; i++) buf_put(b, (uint8_t)(c[i] | (i + 1 == n ? 0x80 : 0)));
    } else {
        fr_vl_write_positive(b, ((int64_t)n << 4) + (1 << 3));    /* full UTF marker */
        for (int i = 0; i < n; i++) {
            if (c[i] <= 0x7F) buf_put(b, (uint8_t)c[i]);
            else if (c[i] > 0x7FF) { buf_put(b, (uint8_t)(0xE0 | (c[i] >> 12 & 0x0F))); buf_put(b, (uint8_t)(0x80 | (c[i] >> 6 & 0x3F))); buf_put(b, (uint8_t)(0x80 | (c[i] & 0x3F))); }
            else { buf_put(b, (uint8_t)(0xC0 | (c[i] >> 6 & 0x1F))); buf_put(b, (uint8_t)(0x80 | (c[i] & 0x3F))); }
        }
    }
}
/* StandardSerializer.writeObjectInternal :286-301: a null flag byte (0 / -1) unless the
 * serializer handles null itself (StringSerializer is a SupportsNullSerializer), then the
 * attribute serializer's write or, for sort keys, writeByteOrder. */
int fr_write_value(fr_buf* b, int dt, int present, int64_t value, int byte_order) {
    if (dt == FR_DT_STRING) {
        if (byte_order) {                                        /* StringSerializer.writeByteOrder :54-67 */
            if (!present) { buf_put(b, 0xFF); return FR_OK; }
            buf_put(b, 0x00);
            uint16_t c[32]; int n = fr_string_of(value, c);
            for (int i = 0; i < n; i++) put_be(b, c[i], 2);      /* CharacterSerializer: the char, big-endian */
            put_be(b, 0, 2);
        } else if (!present) fr_vl_write_positive(b, 0);
        else write_string(b, value);
        return FR_OK;
    }
    if (!present) { buf_put(b, 0xFF); return FR_OK; }
    buf_put(b, 0x00);
    switch (dt) {
    case FR_DT_BYTE: buf_put(b, (uint8_t)((int8_t)value - (-128))); break;          /* ByteSerializer :17-19 */
    case FR_DT_SHORT: put_be(b, (uint16_t)((int16_t)value - (-32768)), 2); break;    /* ShortSerializer :17-19 */
    case FR_DT_CHARACTER: put_be(b, (uint16_t)value, 2); break;                      /* CharacterSerializer: short(c - 2^15) + 2^15 */
    case FR_DT_INTEGER:
        if (byte_order) put_be(b, (uint32_t)((int32_t)value - INT32_MIN), 4);        /* IntegerSerializer :27-34 */
        else fr_vl_write(b, (int32_t)value);                                         /* :20-23 */
        break;
    case FR_DT_LONG: case FR_DT_DATE:                                                /* LongSerializer :20-22, DateSerializer */
        put_be(b, (uint64_t)value - (uint64_t)INT64_MIN, 8); break;
    case FR_DT_FLOAT: {                                                              /* FloatSerializer :33-46 */
        uint32_t u = float_bits(value);
        if (byte_order) { int32_t si = (int32_t)u; si ^= (si >> 31) & 0x7fffffff; u = (uint32_t)si ^ 0x80000000u; }
        put_be(b, u, 4); break;                                  /* NumericUtils.floatToSortableInt */
    }
    case FR_DT_DOUBLE: {                                                             /* DoubleSerializer :33-46 */
        uint64_t u = double_bits(value);
        if (byte_order) { int64_t sl = (int64_t)u; sl ^= (sl >> 63) & 0x7fffffffffffffffLL; u = (uint64_t)sl ^ 0x8000000000000000ULL; }
        put_be(b, u, 8); break;
    }
    case FR_DT_BOOLEAN: buf_put(b, value ? 1 : 0); break;
    default: return FR_E_UNSUPPORTED;
    }
    return FR_OK;
}
static int write_object(fr_buf* b, int dt, int present, int64_t value, int byte_order) {
    return fr_write_value(b, dt, present, value, byte_order);
}
/* StandardSerializer.readObjectInternal :220-233 + the attribute serializers' read /
 * readByteOrder.  d is read through `x` (0xFF inverts: a DESC sort key, EdgeSerializer.java:137).
 * *ival is the value of integral types (Byte..Long, Boolean, Date, Character); other types
 * are skipped (*ival = 0).  *present = 0 on a serialized null. */
static int read_object_x(const uint8_t* d, size_t len, size_t* pos, int dt, int byte_order, uint8_t x,
                         int* present, int64_t* ival) {
#define RD() ((*pos) < len ? (uint8_t)(d[(*pos)++] ^ x) : (uint8_t)((*pos)++, 0))
    *ival = 0;
    if (dt == FR_DT_STRING) {
        if (byte_order) {                                        /* StringSerializer.readByteOrder :40-51 */
            if (*pos >= len) return FR_E_CODEC;
            uint8_t p = RD();
            if (p == 0xFF) { *present = 0; return FR_OK; }
            if (p != 0) return FR_E_CODEC;
            *present = 1;
            for (;;) {
                if (*pos + 2 > len) return FR_E_CODEC;
                uint8_t h = RD(), l = RD();
                if (h == 0 && l == 0) break;
            }
            return FR_OK;
        }
        /* StringSerializer.read :84-135 */
        uint64_t L = 0; uint8_t bb;
        do { if (*pos >= len) return FR_E_CODEC; bb = RD(); L = (L << 7) | (bb & 0x7F); } while (!(bb & 0x80));
        if (L == 0) { *present = 0; return FR_OK; }
        *present = 1;
        uint64_t cid = L & 7; L >>= 3;
        if (cid != 0) { *pos += L; return *pos <= len ? FR_OK : FR_E_CODEC; }   /* compressed: L bytes */
        if ((L & 1) == 0) {
            L >>= 1;
            if (L == 1) return FR_OK;                            /* "" */
            if (L != 2) return FR_E_CODEC;
            do { if (*pos >= len) return FR_E_CODEC; bb = RD(); } while (!(bb & 0x80));
            return FR_OK;
        }
        L >>= 1;
        for (uint64_t i = 0; i < L; i++) {
            if (*pos >= len) return FR_E_CODEC;
            uint8_t c = RD();
            switch (c >> 4) {
            case 12: case 13: RD(); break;
            case 14: RD(); RD(); break;
            default: break;
            }
        }
        return *pos <= len ? FR_OK : FR_E_CODEC;
    }
    if (*pos >= len) return FR_E_CODEC;
    int8_t flag = (int8_t)RD();
    if (flag == -1) { *present = 0; return FR_OK; }
    if (flag != 0) return FR_E_CODEC;
    *present = 1;
    uint64_t u = 0;
    switch (dt) {
    case FR_DT_BYTE: *ival = (int8_t)(RD() + (-128)); break;
    case FR_DT_SHORT: u = RD(); u = (u << 8) | RD(); *ival = (int16_t)(u + (-32768)); break;
    case FR_DT_CHARACTER: u = RD(); u = (u << 8) | RD(); *ival = (int64_t)(uint16_t)u; break;
    case FR_DT_INTEGER:
        if (byte_order) { for (int i = 0; i < 4; i++) u = (u << 8) | RD(); *ival = (int32_t)((uint32_t)u + (uint32_t)INT32_MIN); }
        else {
            uint64_t z = 0; uint8_t bb;
            do { if (*pos >= len) return FR_E_CODEC; bb = RD(); z = (z << 7) | (bb & 0x7F); } while (!(bb & 0x80));
            int64_t l = (z & 1) ? -(int64_t)(z >> 1) : (int64_t)(z >> 1);   /* VariableLong.read zig-zag */
            if (l < INT32_MIN || l > INT32_MAX) return FR_E_CODEC;
            *ival = l;
        }
        break;
    case FR_DT_LONG: case FR_DT_DATE: for (int i = 0; i < 8; i++) u = (u << 8) | RD(); *ival = (int64_t)(u + (uint64_t)INT64_MIN); break;
    case FR_DT_FLOAT: {                                  /* FloatSerializer.read / readByteOrder :33-46 */
        uint32_t u = 0;
        for (int i = 0; i < 4; i++) u = (u << 8) | RD();
        if (byte_order) {                                /* NumericUtils.sortableIntToFloat */
            u ^= 0x80000000u;
            int32_t si = (int32_t)u;
            si ^= (si >> 31) & 0x7fffffff;
            u = (uint32_t)si;
        }
        if (u == 0x80000000u) u = 0;                     /* -0.0f as +0.0f (the product's weight sentinel) */
        *ival = (int32_t)u;                              /* the IEEE bits */
        break;
    }
    case FR_DT_DOUBLE: {                                 /* DoubleSerializer.read / readByteOrder :25-41 */
        for (int i = 0; i < 8; i++) u = (u << 8) | RD();
        if (byte_order) {                                /* LongSerializer.readByteOrder + sortableLongToDouble */
            int64_t sl = (int64_t)(u ^ 0x8000000000000000ULL);
            sl ^= (sl >> 63) & 0x7fffffffffffffffLL;
            u = (uint64_t)sl;
        }
        *ival = (int64_t)u;                              /* the IEEE bits */
        break;
    }
    case FR_DT_BOOLEAN: *ival = RD(); break;
    default: return FR_E_UNSUPPORTED;
    }
#undef RD
    return *pos <= len ? FR_OK : FR_E_CODEC;
}
static int read_object(const uint8_t* d, size_t len, size_t* pos, int dt, int byte_order,
                       int* present, int64_t* ival) {
    return read_object_x(d, len, pos, dt, byte_order, 0, present, ival);
}

int fr_encode_vertex_exists(fr_buf* out, int32_t* value_pos, int64_t relation_id) {
    /* BaseKey.VertexExists (BaseKey.java:27-28): system property key count 1, SINGLE
     * cardinality => constrained & unique: valuePos before value (EdgeSerializer.java:277-281). */
    fr_write_relation_type(out, fr_schema_id(1, 1), 0, 0, 1);
    *value_pos = (int32_t)out->len;
    write_object(out, FR_DT_BOOLEAN, 1, 1, 0);
    fr_vl_write_positive(out, relation_id);
    return FR_OK;
}

int fr_encode_property(fr_buf* out, int32_t* value_pos, int64_t key_id, int datatype,
                       int64_t value, int64_t relation_id) {
    /* user property of SINGLE cardinality: constrained & unique OUT => valuePos before
     * the value, then the relation id (EdgeSerializer.java:270-281). */
    fr_write_relation_type(out, key_id, 0, 0, 0);
    *value_pos = (int32_t)out->len;
    int rc = write_object(out, datatype, 1, value, 0);
    if (rc) return rc;
    fr_vl_write_positive(out, relation_id);
    return FR_OK;
}

int fr_encode_property_f64(fr_buf* out, int32_t* value_pos, int64_t key_id, double value, int64_t relation_id) {
    fr_write_relation_type(out, key_id, 0, 0, 0);                       /* EdgeSerializer.java:270-281 */
    *value_pos = (int32_t)out->len;
    buf_put(out, 0x00);                                                 /* StandardSerializer null flag */
    uint64_t u; memcpy(&u, &value, 8);
    put_be(out, u, 8);
    fr_vl_write_positive(out, relation_id);
    return FR_OK;
}

/* A generic (Object-typed) property key — what DefaultSchemaMaker.makePropertyKey creates for a
 * key the program sets without a schema (dataType(Object.class), DefaultSchemaMaker.java:46-48).
 * AttributeUtil.hasGenericDataType(key) => EdgeSerializer.writePropertyValue :353-356 calls
 * StandardSerializer.writeClassAndObject (:316-322): VariableLong.writePositive of the value
 * class's registration number (registerClassInternal :66-82: Integer 12, Long 13, Double 20),
 * then writeObjectNotNullInternal (:303-314): the class's serializer with NO null flag.
 * value_dt is the value's class; a Double value is passed as its IEEE bits. */
int fr_encode_property_generic(fr_buf* out, int32_t* value_pos, int64_t key_id, int value_dt,
                               int64_t value, int64_t relation_id) {
    int reg;
    switch (value_dt) {
    case FR_DT_INTEGER: reg = 12; break;
    case FR_DT_LONG: reg = 13; break;
    case FR_DT_DOUBLE: reg = 20; break;
    default: return FR_E_UNSUPPORTED;
    }
    fr_write_relation_type(out, key_id, 0, 0, 0);                       /* EdgeSerializer.java:270-281 */
    *value_pos = (int32_t)out->len;
    fr_vl_write_positive(out, (uint64_t)reg);
    if (value_dt == FR_DT_DOUBLE) put_be(out, (uint64_t)value, 8);      /* DoubleSerializer.write: raw bits */
    else {
        const size_t mark = out->len;
        int rc = write_object(out, value_dt, 1, value, 0);
        if (rc) return rc;
        memmove(out->p + mark, out->p + mark + 1, out->len - mark - 1); /* no null flag */
        out->len--;
    }
    fr_vl_write_positive(out, relation_id);
    return FR_OK;
}

int fr_encode_edge(fr_buf* out, int32_t* value_pos, const fr_schema* schema, int64_t type_id,
                   int dir, int64_t other, int64_t relation_id, const fr_prop* props, int nprops) {
    /* EdgeSerializer.writeRelation :222-315 (edge branch :255-266) */
    const fr_edge_type* t = find_type(schema, type_id);
    if (!t) return FR_E_INVALID;
    fr_write_relation_type(out, type_id, 1, dir, 0);
    int mult = t->multiplicity;
    if (mult == FR_MULTI) {
        const size_t key_start = out->len;
        for (int k = 0; k < t->n_sort_key; k++) {                        /* writeInlineTypes KEY */
            int present = 0; int64_t v = 0;
            for (int j = 0; j < nprops; j++) if (props[j].key_id == t->sort_key_ids[k]) { present = 1; v = props[j].value; }
            int rc = write_object(out, key_datatype(schema, t->sort_key_ids[k]), present, v, 1);
            if (rc) return rc;
        }
        if (t->sort_order == FR_DESC)                                    /* getStaticBufferFlipBytes :311-313 */
            for (size_t i = key_start; i < out->len; i++) out->p[i] = (uint8_t)~out->p[i];
        fr_vl_write_positive_backward(out, other);
        fr_vl_write_positive_backward(out, relation_id);
        *value_pos = (int32_t)out->len;
    } else if (is_unique(mult, dir)) {
        *value_pos = (int32_t)out->len;
        fr_vl_write_positive(out, other);
        fr_vl_write_positive(out, relation_id);
    } else {
        fr_vl_write_positive_backward(out, other);
        *value_pos = (int32_t)out->len;
        fr_vl_write_positive(out, relation_id);
    }
    for (int k = 0; k < t->n_signature; k++) {                           /* signature :285 */
        int present = 0; int64_t v = 0;
        for (int j = 0; j < nprops; j++) if (props[j].key_id == t->signature_ids[k]) { present = 1; v = props[j].value; }
        int rc = write_object(out, key_datatype(schema, t->signature_ids[k]), present, v, 0);
        if (rc) return rc;
    }
    /* remaining properties, sorted by key id (:287-308) */
    int64_t rem[64]; int nrem = 0;
    for (int j = 0; j < nprops && nrem < 64; j++) {
        int64_t id = props[j].key_id, skip = 0;
        if (mult == FR_MULTI) for (int k = 0; k < t->n_sort_key; k++) skip |= t->sort_key_ids[k] == id;
        for (int k = 0; k < t->n_signature; k++) skip |= t->signature_ids[k] == id;
        if (!skip) rem[nrem++] = id;
    }
    for (int a = 1; a < nrem; a++) for (int c = a; c > 0 && rem[c - 1] > rem[c]; c--) { int64_t x = rem[c]; rem[c] = rem[c - 1]; rem[c - 1] = x; }
    for (int a = 0; a < nrem; a++) {
        int64_t v = 0;
        for (int j = 0; j < nprops; j++) if (props[j].key_id == rem[a]) v = props[j].value;
        fr_vl_write_positive(out, (int64_t)((uint64_t)rem[a] >> 4));    /* writeInlineRelationType, IDHandler :135-138 */
        int rc = write_object(out, key_datatype(schema, rem[a]), 1, v, 0);
        if (rc) return rc;
    }
    return FR_OK;
}

int fr_weight_datatype_ok(int dt) {
    return dt == FR_DT_INTEGER || dt == FR_DT_BYTE || dt == FR_DT_SHORT || dt == FR_DT_CHARACTER ||
           dt == FR_DT_BOOLEAN || dt == FR_DT_FLOAT || dt == FR_DT_LONG || dt == FR_DT_DOUBLE;
}

int fr_decode_edge(const uint8_t* d, size_t len, size_t value_pos, const fr_schema* schema,
                   int64_t weight_key, int64_t* type_id, int* dir, int64_t* other_id,
                   int64_t* relation_id, int* has_weight, int64_t* weight) {
    /* EdgeSerializer.parseRelation :73-166 (edge branch :90-110, properties :138-158) */
    size_t pos = 0;
    int is_edge;
    if (len == 0 || value_pos > len) return FR_E_CODEC;
    int rc = fr_read_relation_type(d, &pos, type_id, &is_edge, dir);
    if (rc) return rc;
    if (!is_edge) return FR_E_CODEC;
    const fr_edge_type* t = find_type(schema, *type_id);
    if (!t) return FR_E_CODEC;                                           /* tx.getExistingRelationType */
    int mult = t->multiplicity;
    size_t props_pos;
    if (mult != FR_MULTI) {
        if (is_unique(mult, *dir)) {
            *other_id = fr_vl_read_positive(d, &pos);
        } else {
            size_t p = value_pos;
            *other_id = fr_vl_read_positive_backward(d, &p);
            pos = value_pos;
        }
        *relation_id = fr_vl_read_positive(d, &pos);
        props_pos = pos;
    } else {
        size_t p = value_pos;
        *relation_id = fr_vl_read_positive_backward(d, &p);
        *other_id = fr_vl_read_positive_backward(d, &p);
        props_pos = value_pos;
    }
    *has_weight = 0;
    if (weight_key == 0) return FR_OK;
    /* The weight: an integral key that fits 32 bits, or a Float (its IEEE bits).
     * ShortestDistance itself casts to Integer (ShortestDistanceVertexProgram.java:53):
     * fr_shortest_distance rejects the others (a ClassCastException in the reference). */
    if (!fr_weight_datatype_ok(key_datatype(schema, weight_key))) return FR_E_UNSUPPORTED;
    if (mult == FR_MULTI) {                                              /* sort key :130-140 */
        size_t kp = pos;                                                 /* startKeyPos: after the type */
        const uint8_t x = t->sort_order == FR_DESC ? 0xFF : 0x00;        /* in.subrange(keyLength, true) */
        for (int k = 0; k < t->n_sort_key; k++) {
            int present; int64_t v = 0;
            rc = read_object_x(d, value_pos, &kp, key_datatype(schema, t->sort_key_ids[k]), 1, x, &present, &v);
            if (rc) return rc;
            if (t->sort_key_ids[k] == weight_key) { *has_weight = present; *weight = v; return FR_OK; }
        }
    }
    pos = props_pos;
    for (int k = 0; k < t->n_signature; k++) {                           /* readInlineTypes SIGNATURE */
        int present; int64_t v = 0;
        rc = read_object(d, len, &pos, key_datatype(schema, t->signature_ids[k]), 0, &present, &v);
        if (rc) return rc;
        if (t->signature_ids[k] == weight_key) { *has_weight = present; *weight = v; return FR_OK; }
    }
    while (pos < len) {                                                  /* remaining :147-152 */
        int64_t kid = (fr_vl_read_positive(d, &pos) << 4) | 5;           /* readInlineRelationType */
        int present; int64_t v = 0;
        rc = read_object(d, len, &pos, key_datatype(schema, kid), 0, &present, &v);
        if (rc) return rc;
        if (kid == weight_key) { *has_weight = present; *weight = v; return FR_OK; }
    }
    return FR_OK;
}

/* ===================================================================== graph */
struct fr_graph {
    int64_t n;
    int64_t* titan_id;        /* n, row order                                   */
    int64_t* eoff;            /* n+1: kept user-edge entries of each row          */
    int64_t* other;           /* E: other vertex Titan id                         */
    uint8_t* edir;            /* E: 0 OUT, 1 IN                                   */
    uint8_t* has_w;           /* E                                                */
    int64_t* w;               /* E (Long / Double keys: the value / its IEEE bits) */
    /* FulgoraVertexMemory's NonBlockingHashMapLong<VertexState>: Titan id -> index */
    int64_t* hkeys; int64_t* hvals; uint64_t hmask;
    /* Vertex cuts: pv[v] = 1 for a canonical partitioned vertex.  Its canonical row's
     * entries are [eoff[v], eoff[v+1]); every other representative row r of it (in scan
     * order) is xr_beg[j]..xr_end[j] for j in [xr_off[v], xr_off[v+1]). NULL if none. */
    uint8_t* pv;
    int64_t* xr_off; int64_t* xr_beg; int64_t* xr_end;
    /* Optional memo of lookup(other[k]) per entry (fr_resolve): the hash probe is a pure
     * function of the loaded graph, so caching it changes no result, only the oracle's speed
     * on the full-size parity tests.  NULL = probe the hash map per entry, as the reference. */
    int64_t* oidx;
    int64_t nent;             /* entries stored in other/edir/has_w/w                */
    int32_t wdt;              /* datatype of the weight key (0: Integer / none)       */
};

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
static void build_hash(fr_graph* g) {
    uint64_t cap = 16; while (cap < (uint64_t)g->n * 2) cap <<= 1;
    g->hmask = cap - 1;
    g->hkeys = (int64_t*)malloc(cap * sizeof(int64_t));
    g->hvals = (int64_t*)malloc(cap * sizeof(int64_t));
    for (uint64_t i = 0; i < cap; i++) g->hkeys[i] = INT64_MIN;
    for (int64_t v = 0; v < g->n; v++) {
        uint64_t h = mix64((uint64_t)g->titan_id[v]) & g->hmask;
        while (g->hkeys[h] != INT64_MIN && g->hkeys[h] != g->titan_id[v]) h = (h + 1) & g->hmask;
        g->hkeys[h] = g->titan_id[v]; g->hvals[h] = v;
    }
}
static inline int64_t lookup(const fr_graph* g, int64_t id) {            /* vertexStates.get :49-58 */
    uint64_t h = mix64((uint64_t)id) & g->hmask;
    for (;;) {
        int64_t k = g->hkeys[h];
        if (k == id) return g->hvals[h];
        if (k == INT64_MIN) return -1;                                   /* EMPTY_STATE */
        h = (h + 1) & g->hmask;
    }
}

/* The executor's per-entry neighbour lookup (VertexMemoryHandler.java:89 -> getMessage). */
static inline int64_t entry_vertex(const fr_graph* g, int64_t k) {
    return g->oidx ? g->oidx[k] : lookup(g, g->other[k]);
}

void fr_free(fr_graph* g) {
    if (!g) return;
    free(g->oidx);
    free(g->titan_id); free(g->eoff); free(g->other); free(g->edir); free(g->has_w); free(g->w);
    free(g->hkeys); free(g->hvals);
    free(g->pv); free(g->xr_off); free(g->xr_beg); free(g->xr_end); free(g);
}
int64_t fr_num_vertices(const fr_graph* g) { return g->n; }
void fr_vertex_ids(const fr_graph* g, int64_t* out) { memcpy(out, g->titan_id, g->n * sizeof(int64_t)); }
/* Rows of vertex v: 0 = its own (canonical) row, 1.. = its other representative rows. */
static inline int64_t nrows_of(const fr_graph* g, int64_t v) {
    return 1 + (g->xr_off ? g->xr_off[v + 1] - g->xr_off[v] : 0);
}
static inline void row_range(const fr_graph* g, int64_t v, int64_t i, int64_t* b, int64_t* e) {
    if (i == 0) { *b = g->eoff[v]; *e = g->eoff[v + 1]; return; }
    int64_t j = g->xr_off[v] + i - 1;
    *b = g->xr_beg[j]; *e = g->xr_end[j];
}
int64_t fr_num_entries(const fr_graph* g) {
    int64_t e = 0;
    for (int64_t v = 0; v < g->n; v++)
        for (int64_t i = 0; i < nrows_of(g, v); i++) { int64_t b, x; row_range(g, v, i, &b, &x); e += x - b; }
    return e;
}

/* Decode the kept user-edge entries of one row into g->other/edir/has_w/w from index *e. */
static int decode_row_entries(const fr_rows* rows, int64_t r, const fr_schema* schema, const fr_load_opts* opts,
                              int64_t limit, fr_graph* g, int64_t* e, fr_load_stats* st) {
    int pb = opts->partition_bits;
    int typed = opts->n_labels > 0;
    const uint8_t* base = rows->entry_bytes + rows->row_byte_begin[r];
    int64_t e0 = rows->row_entry_begin[r], e1 = rows->row_entry_begin[r + 1];
    /* user-edge slice: column first byte in [0x60, 0x80) (IDHandler.getBounds :158-179) */
    int64_t cnt = 0, first = -1;
    for (int64_t k = e0; k < e1; k++) {
        int64_t start = k == e0 ? 0 : (int64_t)((uint64_t)rows->entry_limit_valpos[k - 1] >> 32);
        uint8_t c0 = base[start];
        if (c0 >= 0x60 && c0 < 0x80) { if (first < 0) first = k; cnt++; }
    }
    if (limit != INT64_MAX && cnt >= limit) st->truncated_results++;    /* VertexJobConverter :125 */
    int64_t keep = cnt < limit ? cnt : limit;
    for (int64_t k = first; k >= 0 && k < first + keep; k++) {
        int64_t start = k == e0 ? 0 : (int64_t)((uint64_t)rows->entry_limit_valpos[k - 1] >> 32);
        int64_t end = (int64_t)((uint64_t)rows->entry_limit_valpos[k] >> 32);
        int64_t vpos = rows->entry_limit_valpos[k] & 0x7FFFFFFF;
        int64_t tid, oid, rid, wv = 0; int dr, hw;
        int rc = fr_decode_edge(base + start, (size_t)(end - start), (size_t)vpos, schema,
                                opts->weight_key, &tid, &dr, &oid, &rid, &hw, &wv);
        if (rc) return rc;
        if (typed) {
            int ok = 0; for (int j = 0; j < opts->n_labels; j++) ok |= opts->label_ids[j] == tid;
            if (!ok) continue;
        }
        /* messages are looked up by canonical id (VertexMemoryHandler.java:89) */
        if (fr_is_partitioned(oid, pb)) oid = fr_canonical_vertex_id(oid, pb);
        g->other[*e] = oid; g->edir[*e] = (uint8_t)dr; g->has_w[*e] = (uint8_t)hw; g->w[*e] = wv;
        (*e)++;
    }
    return FR_OK;
}

int fr_load_rows(const fr_rows* rows, const fr_schema* schema, const fr_load_opts* opts,
                 fr_graph** out, fr_load_stats* stats) {
    /* VertexJobConverter.process/getKeyFilter/isGhostVertex (VertexJobConverter.java:109-171)
     * + slice [0x60,0x80) with the QueryContainer limit (QueryContainer.java:110-134).
     * Vertex cuts: a non-canonical representative row skips the ghost check (:132); its
     * messages are folded into the canonical vertex's aggregate (VertexProgramScanJob.java
     * :76-92), which only executes if the canonical row was processed (setLoadedProperties
     * :78-81; otherwise GHOTST_PARTITION_VERTEX, PartitionedVertexProgramExecutor.java:53-56). */
    fr_load_stats st; memset(&st, 0, sizeof st);
    int pb = opts->partition_bits;
    int64_t nr = rows->nrows;
    fr_graph* g = (fr_graph*)calloc(1, sizeof(fr_graph));
    int64_t total = rows->row_entry_begin[nr];
    g->titan_id = (int64_t*)malloc((nr + 1) * sizeof(int64_t));
    g->eoff = (int64_t*)malloc((nr + 1) * sizeof(int64_t));
    g->pv = (uint8_t*)calloc(nr + 1, 1);
    g->other = (int64_t*)malloc((total + 1) * sizeof(int64_t));
    g->edir = (uint8_t*)malloc(total + 1);
    g->has_w = (uint8_t*)malloc(total + 1);
    g->w = (int64_t*)malloc((total + 1) * sizeof(int64_t));
    int typed = opts->n_labels > 0;
    int64_t limit = (opts->apply_cap && !typed && opts->scope != FR_SCOPE_BOTH_E) ? opts->hard_query_limit : INT64_MAX;
    /* pass 1: which rows execute (0 = filtered, 1 = vertex row, 2 = representative row) */
    int8_t* kind = (int8_t*)calloc(nr + 1, 1);
    int64_t* rid = (int64_t*)malloc((nr + 1) * sizeof(int64_t));
    int64_t n = 0, nrep = 0;
    for (int64_t r = 0; r < nr; r++) {
        int64_t vid = fr_key_id(rows->row_keys[r], pb);
        if (fr_is_invisible(vid)) { st.skipped_rows++; continue; }       /* getKeyFilter :156-162 */
        int64_t sfx = vid & 7;
        if (sfx != 0 && sfx != 2 && sfx != 4) { fr_free(g); free(kind); free(rid); return FR_E_CODEC; }  /* getUserVertexIDType */
        const uint8_t* base = rows->entry_bytes + rows->row_byte_begin[r];
        if (rows->row_entry_begin[r + 1] <= rows->row_entry_begin[r]) { fr_free(g); free(kind); free(rid); return FR_E_CODEC; }
        if (sfx == 2 && vid != fr_canonical_vertex_id(vid, pb)) {        /* isGhostVertex :132 */
            kind[r] = 2; rid[r] = fr_canonical_vertex_id(vid, pb); nrep++;
            continue;
        }
        {   /* ghost check: first entry must be VertexExists (:131-137) */
            size_t pos = 0; int64_t tid; int ie, dr;
            if (fr_read_relation_type(base, &pos, &tid, &ie, &dr)) { fr_free(g); free(kind); free(rid); return FR_E_CODEC; }
            if (ie || tid != fr_schema_id(1, 1)) { st.ghost_vertices++; continue; }
        }
        kind[r] = 1; rid[r] = vid;
        g->titan_id[n] = vid;
        g->pv[n] = sfx == 2;
        st.partitioned_vertices += sfx == 2;
        n++;
    }
    g->n = n;
    build_hash(g);
    /* pass 2: entries of vertex rows, in row order; then the representative rows */
    int64_t e = 0, v = 0;
    g->eoff[0] = 0;
    for (int64_t r = 0; r < nr; r++) {
        if (kind[r] != 1) continue;
        int rc = decode_row_entries(rows, r, schema, opts, limit, g, &e, &st);
        if (rc) { fr_free(g); free(kind); free(rid); return rc; }
        g->eoff[++v] = e;
    }
    if (nrep) {
        int64_t* xv = (int64_t*)malloc(nrep * sizeof(int64_t));
        int64_t* xb = (int64_t*)malloc(nrep * sizeof(int64_t));
        int64_t* xe = (int64_t*)malloc(nrep * sizeof(int64_t));
        int64_t j = 0;
        for (int64_t r = 0; r < nr; r++) {
            if (kind[r] != 2) continue;
            int64_t owner = lookup(g, rid[r]);
            if (owner < 0) { st.ghost_partition_rows++; continue; }
            xv[j] = owner; xb[j] = e;
            int rc = decode_row_entries(rows, r, schema, opts, limit, g, &e, &st);
            if (rc) { free(xv); free(xb); free(xe); fr_free(g); free(kind); free(rid); return rc; }
            xe[j] = e; j++;
        }
        st.partition_rows = j;
        /* per-vertex CSR of representative rows, scan order kept */
        g->xr_off = (int64_t*)calloc(n + 1, sizeof(int64_t));
        g->xr_beg = (int64_t*)malloc((j + 1) * sizeof(int64_t));
        g->xr_end = (int64_t*)malloc((j + 1) * sizeof(int64_t));
        for (int64_t i = 0; i < j; i++) g->xr_off[xv[i] + 1]++;
        for (int64_t u = 0; u < n; u++) g->xr_off[u + 1] += g->xr_off[u];
        int64_t* pos = (int64_t*)malloc((n + 1) * sizeof(int64_t));
        memcpy(pos, g->xr_off, (n + 1) * sizeof(int64_t));
        for (int64_t i = 0; i < j; i++) { int64_t p = pos[xv[i]]++; g->xr_beg[p] = xb[i]; g->xr_end[p] = xe[i]; }
        free(pos); free(xv); free(xb); free(xe);
    }
    free(kind); free(rid);
    st.num_entries = e;
    g->nent = e;
    g->wdt = opts->weight_key ? key_datatype(schema, opts->weight_key) : 0;
    *out = g;
    if (stats) *stats = st;
    return FR_OK;
}

int fr_load_adjacency(int64_t n, const int64_t* titan_ids, const int64_t* off, const int64_t* mid,
                      const int32_t* adj, const int32_t* w, fr_graph** out) {
    fr_graph* g = (fr_graph*)calloc(1, sizeof(fr_graph));
    int64_t E = off[n];
    g->n = n;
    g->titan_id = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    g->pv = (uint8_t*)calloc(n + 1, 1);
    g->eoff = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    g->other = (int64_t*)malloc((E + 1) * sizeof(int64_t));
    g->edir = (uint8_t*)malloc(E + 1);
    g->has_w = (uint8_t*)malloc(E + 1);
    g->w = (int64_t*)malloc((E + 1) * sizeof(int64_t));
    memcpy(g->titan_id, titan_ids, n * sizeof(int64_t));
    memcpy(g->eoff, off, (n + 1) * sizeof(int64_t));
    for (int64_t v = 0; v < n; v++)
        for (int64_t k = off[v]; k < off[v + 1]; k++) {
            g->other[k] = titan_ids[adj[k]];
            g->edir[k] = k >= mid[v];
            g->has_w[k] = w != NULL;
            g->w[k] = w ? w[k] : 0;
        }
    g->nent = E;
    build_hash(g);
    *out = g;
    return FR_OK;
}

int fr_load_edges_capped(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* w,
                         const int64_t* titan_ids, int64_t hard_limit, int64_t* truncated, fr_graph** out) {
    /* Rows as the commit path writes them (StandardTitanGraph.java:564-591): every edge
     * u->v gives an OUT entry on row u and an IN entry on row v; within a row OUT entries
     * precede IN entries and each run is ordered by (other id, relation id = edge index).
     * hard_limit > 0 restates the preload cap of an untyped single-direction scope: the
     * row's user-edge slice is returned in column order and cut at the limit
     * (QueryContainer.java:28,122; ColumnValueStore.getSlice :59), and a row with at least
     * `limit` entries counts as truncated (VertexJobConverter.java:125). */
    fr_graph* g = (fr_graph*)calloc(1, sizeof(fr_graph));
    g->n = n;
    g->titan_id = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    g->pv = (uint8_t*)calloc(n + 1, 1);
    g->eoff = (int64_t*)calloc(n + 1, sizeof(int64_t));
    int64_t E = 2 * m;
    g->other = (int64_t*)malloc((E + 1) * sizeof(int64_t));
    g->edir = (uint8_t*)malloc(E + 1);
    g->has_w = (uint8_t*)malloc(E + 1);
    g->w = (int64_t*)malloc((E + 1) * sizeof(int64_t));
    for (int64_t v = 0; v < n; v++) g->titan_id[v] = titan_ids[v];
    int64_t* outc = (int64_t*)calloc(n + 1, sizeof(int64_t));
    for (int64_t k = 0; k < m; k++) { outc[src[k]]++; g->eoff[src[k] + 1]++; g->eoff[dst[k] + 1]++; }
    for (int64_t v = 0; v < n; v++) g->eoff[v + 1] += g->eoff[v];
    int64_t* po = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    int64_t* pi = (int64_t*)malloc((n + 1) * sizeof(int64_t));
    for (int64_t v = 0; v < n; v++) { po[v] = g->eoff[v]; pi[v] = g->eoff[v] + outc[v]; }
    /* counting sort by neighbour keeps edge-index order among equal neighbours */
    int64_t* bucket = (int64_t*)calloc(n + 1, sizeof(int64_t));
    int64_t* order = (int64_t*)malloc((m + 1) * sizeof(int64_t));
    for (int pass = 0; pass < 2; pass++) {
        const int32_t* key = pass == 0 ? dst : src;      /* neighbour of the OUT / IN entry */
        const int32_t* own = pass == 0 ? src : dst;
        memset(bucket, 0, (n + 1) * sizeof(int64_t));
        for (int64_t k = 0; k < m; k++) bucket[key[k] + 1]++;
        for (int64_t v = 0; v < n; v++) bucket[v + 1] += bucket[v];
        for (int64_t k = 0; k < m; k++) order[bucket[key[k]]++] = k;
        for (int64_t j = 0; j < m; j++) {
            int64_t k = order[j];
            int64_t p = pass == 0 ? po[own[k]]++ : pi[own[k]]++;
            g->other[p] = titan_ids[key[k]];
            g->edir[p] = (uint8_t)pass;
            g->has_w[p] = w != NULL;
            g->w[p] = w ? w[k] : 0;
        }
    }
    free(outc); free(po); free(pi); free(bucket); free(order);
    int64_t cut = 0;
    if (hard_limit > 0) {                               /* compact rows to their first `limit` entries */
        int64_t wpos = 0, beg = 0;
        for (int64_t v = 0; v < n; v++) {
            int64_t end = g->eoff[v + 1], cnt = end - beg;
            if (cnt >= hard_limit) cut++;
            int64_t keep = cnt < hard_limit ? cnt : hard_limit;
            for (int64_t k = beg; k < beg + keep; k++, wpos++) {
                g->other[wpos] = g->other[k]; g->edir[wpos] = g->edir[k];
                g->has_w[wpos] = g->has_w[k]; g->w[wpos] = g->w[k];
            }
            beg = end;
            g->eoff[v + 1] = wpos;
        }
    }
    if (truncated) *truncated = cut;
    g->nent = g->eoff[n];
    build_hash(g);
    *out = g;
    return FR_OK;
}

int fr_load_edges(int64_t n, int64_t m, const int32_t* src, const int32_t* dst, const int32_t* w,
                  const int64_t* titan_ids, fr_graph** out) {
    return fr_load_edges_capped(n, m, src, dst, w, titan_ids, 0, NULL, out);
}

typedef struct { fr_graph* g; int64_t lo, hi; } resolve_t;
static void* resolve_range(void* a) {
    resolve_t* r = (resolve_t*)a;
    for (int64_t k = r->lo; k < r->hi; k++) r->g->oidx[k] = lookup(r->g, r->g->other[k]);
    return NULL;
}
int fr_resolve(fr_graph* g, int threads) {
    if (g->oidx) return FR_OK;
    g->oidx = (int64_t*)malloc((g->nent + 1) * sizeof(int64_t));
    if (!g->oidx) return FR_E_INVALID;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256]; resolve_t rt[256];
    for (int i = 0; i < threads; i++) {
        rt[i].g = g; rt[i].lo = g->nent * i / threads; rt[i].hi = g->nent * (i + 1) / threads;
        pthread_create(&th[i], NULL, resolve_range, &rt[i]);
    }
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    return FR_OK;
}

int64_t fr_export(const fr_graph* g, int64_t* off, int64_t* mid, int32_t* adj, int32_t* w) {
    /* dense form with OUT entries first within each row (stable); entries whose other
     * endpoint is not an executed vertex are dropped: they can never carry a message
     * (absent VertexState => EMPTY_STATE => null, FulgoraVertexMemory.java:49-58).
     * A vertex cut exports the union of its representative rows (canonical row first). */
    int64_t e = 0;
    off[0] = 0;
    for (int64_t v = 0; v < g->n; v++) {
        for (int pass = 0; pass < 2; pass++) {
            if (pass == 1) mid[v] = e;
            for (int64_t i = 0; i < nrows_of(g, v); i++) {
                int64_t kb, ke; row_range(g, v, i, &kb, &ke);
                for (int64_t k = kb; k < ke; k++) {
                    if (g->edir[k] != pass) continue;
                    int64_t o = entry_vertex(g, k);
                    if (o < 0) continue;
                    adj[e] = (int32_t)o;
                    if (w) w[e] = g->has_w[k] ? (int32_t)g->w[k] : INT32_MIN;
                    e++;
                }
            }
        }
        off[v + 1] = e;
    }
    return e;
}

/* ===================================================================== executor */
/* One superstep = every vertex executes (VertexProgramScanJob.process :71-97), fanned
 * out over `threads` workers (StandardScannerExecutor processors :235-288). */
typedef struct {
    const fr_graph* g; int64_t lo, hi; void* prog; void (*fn)(void*, const fr_graph*, int64_t, int64_t);
} task_t;
static void* run_task(void* a) { task_t* t = (task_t*)a; t->fn(t->prog, t->g, t->lo, t->hi); return NULL; }
static void superstep(const fr_graph* g, int threads, void* prog, void (*fn)(void*, const fr_graph*, int64_t, int64_t)) {
    if (threads < 1) threads = 1;
    if (threads == 1 || g->n < 1024) { fn(prog, g, 0, g->n); return; }
    pthread_t th[256]; task_t tk[256];
    if (threads > 256) threads = 256;
    for (int i = 0; i < threads; i++) {
        tk[i].g = g; tk[i].prog = prog; tk[i].fn = fn;
        tk[i].lo = g->n * i / threads; tk[i].hi = g->n * (i + 1) / threads;
        pthread_create(&th[i], NULL, run_task, &tk[i]);
    }
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
}

/* Reversed scope selection (FulgoraUtil.getReverseTraversal :49-62, reverseDirection :57):
 * scope inE -> receiver walks its OUT entries; outE -> IN entries; bothE -> all. */
static inline int take(int scope, uint8_t edir) {
    if (scope == FR_SCOPE_BOTH_E) return 1;
    return scope == FR_SCOPE_IN_E ? edir == 0 : edir == 1;
}

/* ---- ShortestDistanceVertexProgram (tmain/olap/ShortestDistanceVertexProgram.java:96-130) ---- */
typedef struct {
    int scope, weighted, iteration;
    int64_t seed;
    int64_t* dist;               /* property DISTANCE (immediate, VertexState.setProperty)      */
    int64_t* prev; int64_t* cur; /* double-buffered Local messages (VertexState :55-89)        */
    volatile int failed;
    volatile int sent;           /* any message sent this superstep */
} sd_t;
/* The messages one row receives on the scope, reduced with min: execute()'s reduce
 * (:109-110) for a vertex row, ShortestDistanceMessageCombiner (min, :17) for a
 * representative row of a vertex cut (VertexProgramScanJob.java:82-90). */
static int64_t sd_row_min(sd_t* s, const fr_graph* g, int64_t kb, int64_t ke) {
    int64_t best = FR_ABSENT;
    for (int64_t k = kb; k < ke; k++) {
        if (!take(s->scope, g->edir[k])) continue;
        int64_t o = entry_vertex(g, k);
        if (o < 0) continue;
        int64_t m = s->prev[o];
        if (m == FR_ABSENT) continue;                                    /* filter(m != null) */
        int64_t wt = 1;
        if (s->weighted) {
            if (!g->has_w[k]) { s->failed = 1; continue; }               /* edge.value(weight) throws */
            wt = g->w[k];
        }
        int64_t c = (int64_t)((uint64_t)m + (uint64_t)wt);               /* Long + Integer, Java wrap */
        if (best == FR_ABSENT || c < best) best = c;
    }
    return best;
}
static void sd_exec(void* p, const fr_graph* g, int64_t lo, int64_t hi) {
    sd_t* s = (sd_t*)p;
    for (int64_t v = lo; v < hi; v++) {
        if (s->iteration == 0) {                                         /* :97-104 */
            if (g->titan_id[v] == s->seed) { s->dist[v] = 0; s->cur[v] = 0; s->sent = 1; }
            continue;
        }
        int64_t best = FR_ABSENT;
        if (!g->pv[v]) {
            best = sd_row_min(s, g, g->eoff[v], g->eoff[v + 1]);         /* reduce(min).orElse(null) :109-110 */
        } else {
            /* vertex cut: every representative row's combined message is aggregated with the
             * combiner (FulgoraVertexMemory.aggregateMessage :138-140); execute() then runs once
             * after the scan and receives only the aggregate (PartitionedVertexProgramExecutor
             * :88-95, VertexMemoryHandler.Partition :126-135). */
            for (int64_t i = 0; i < nrows_of(g, v); i++) {
                int64_t kb, ke; row_range(g, v, i, &kb, &ke);
                int64_t m = sd_row_min(s, g, kb, ke);
                if (m != FR_ABSENT && (best == FR_ABSENT || m < best)) best = m;
            }
        }
        if (best == FR_ABSENT) continue;                                 /* :112-113 */
        if (s->dist[v] == FR_ABSENT || s->dist[v] > best) {             /* :117-122 */
            s->dist[v] = best; s->cur[v] = best; s->sent = 1;
        }
    }
}
int fr_shortest_distance(const fr_graph* g, int64_t seed, int max_depth, int scope, int weighted,
                         int threads, int64_t* dist_out, int* iterations_out) {
    /* edge.<Integer>value(weight) (ShortestDistanceVertexProgram.java:53): another weight
     * datatype is a ClassCastException in the reference */
    if (weighted && g->wdt != 0 && g->wdt != FR_DT_INTEGER) return FR_E_UNSUPPORTED;
    sd_t s; memset(&s, 0, sizeof s);
    s.scope = scope; s.weighted = weighted; s.seed = seed;
    s.dist = dist_out;
    s.prev = (int64_t*)malloc((g->n + 1) * sizeof(int64_t));
    s.cur = (int64_t*)malloc((g->n + 1) * sizeof(int64_t));
    for (int64_t v = 0; v < g->n; v++) s.dist[v] = s.prev[v] = s.cur[v] = FR_ABSENT;
    int it;
    for (it = 0;; it++) {                                                /* FulgoraGraphComputer :151-189 */
        s.iteration = it;
        s.sent = 0;
        superstep(g, threads, &s, sd_exec);
        if (s.failed) { free(s.prev); free(s.cur); return FR_E_PROGRAM; }
        int64_t* t = s.prev; s.prev = s.cur; s.cur = t;                  /* completeIteration: prev=cur, cur=null */
        for (int64_t v = 0; v < g->n; v++) s.cur[v] = FR_ABSENT;
        if (it >= max_depth) break;                                      /* terminate :128-130 */
        /* No message was sent: every later superstep receives nothing and changes nothing
         * (:106-113), so skipping them is exact; the reported iteration stays maxDepth. */
        if (!s.sent) { it = max_depth; break; }
    }
    if (iterations_out) *iterations_out = it;                            /* FulgoraMemory.complete :73-76 */
    free(s.prev); free(s.cur);
    return FR_OK;
}

/* ---- PageRankVertexProgram (tmain/olap/PageRankVertexProgram.java:75-100) ---- */
typedef struct {
    int iteration; double alpha; int64_t N;
    double* pr; double* edge_count;
    /* two scopes (outE, inE): VertexState keeps Object[2]; NaN = null message */
    double* prev_out; double* prev_in; double* cur_out; double* cur_in;
    volatile int failed;
} pr_t;
/* One scope's non-null messages on entries [kb,ke) of a row: sum added to *sum in entry
 * order, count returned.  sel = the entry direction the reversed scope walks. */
static int64_t pr_row(const fr_graph* g, const double* prev, int sel, int64_t kb, int64_t ke, double* sum) {
    int64_t cnt = 0;
    for (int64_t k = kb; k < ke; k++) {
        if (g->edir[k] != sel) continue;
        int64_t o = entry_vertex(g, k);
        if (o < 0) continue;
        double m = prev[o];
        if (isnan(m)) continue;
        *sum = *sum + m;
        cnt++;
    }
    return cnt;
}
static void pr_exec(void* p, const fr_graph* g, int64_t lo, int64_t hi) {
    pr_t* s = (pr_t*)p;
    for (int64_t v = lo; v < hi; v++) {
        if (s->iteration == 0) { s->cur_in[v] = 1.0; continue; }         /* :76-77 sendMessage(inE, 1) */
        /* receiveMessages(): concat(inE stream, outE stream) (VertexMemoryHandler :95-102);
         * reduce(0D, a+b) sequentially in that order. */
        double sum = 0.0;
        if (!g->pv[v]) {
            pr_row(g, s->prev_in, 0, g->eoff[v], g->eoff[v + 1], &sum);  /* inE scope: walk OUT entries */
            pr_row(g, s->prev_out, 1, g->eoff[v], g->eoff[v + 1], &sum); /* outE scope: walk IN entries */
        } else {
            /* vertex cut: PageRankVertexProgram has no combiner, so FulgoraUtil's
             * ThrowingCombiner (:80-91) throws as soon as two messages of one scope meet,
             * in one row (VertexProgramScanJob.java:84-87) or across rows
             * (VertexState.addMessage :63-78); the failed row aborts the job
             * (FulgoraGraphComputer.java:165-168).  One message per scope passes through. */
            for (int sc = 0; sc < 2; sc++) {
                int64_t tot = 0; double agg = 0.0;
                for (int64_t i = 0; i < nrows_of(g, v); i++) {
                    int64_t kb, ke; row_range(g, v, i, &kb, &ke);
                    tot += pr_row(g, sc == 0 ? s->prev_in : s->prev_out, sc == 0 ? 0 : 1, kb, ke, &agg);
                }
                if (tot > 1) { s->failed = 1; break; }
                sum = sum + agg;
            }
        }
        if (s->iteration == 1) {                                         /* :78-83 */
            double init = 1.0 / (double)s->N;
            s->pr[v] = init; s->edge_count[v] = sum;
            s->cur_out[v] = init / sum;
        } else {                                                         /* :84-89 */
            double npr = (s->alpha * sum) + ((1.0 - s->alpha) / (double)s->N);
            s->pr[v] = npr;
            s->cur_out[v] = npr / s->edge_count[v];
        }
    }
}
int fr_pagerank(const fr_graph* g, double alpha, int64_t vertex_count, int max_iterations,
                int threads, double* pr_out, int* iterations_out) {
    pr_t s; memset(&s, 0, sizeof s);
    s.alpha = alpha; s.N = vertex_count; s.pr = pr_out;
    size_t nb = (g->n + 1) * sizeof(double);
    s.edge_count = (double*)malloc(nb);
    s.prev_out = (double*)malloc(nb); s.prev_in = (double*)malloc(nb);
    s.cur_out = (double*)malloc(nb); s.cur_in = (double*)malloc(nb);
    for (int64_t v = 0; v < g->n; v++) {
        pr_out[v] = NAN; s.edge_count[v] = NAN;
        s.prev_out[v] = s.prev_in[v] = s.cur_out[v] = s.cur_in[v] = NAN;
    }
    int it;
    for (it = 0;; it++) {
        s.iteration = it;
        superstep(g, threads, &s, pr_exec);
        if (s.failed) {
            free(s.edge_count); free(s.prev_out); free(s.prev_in); free(s.cur_out); free(s.cur_in);
            return FR_E_PROGRAM;
        }
        double* t;
        t = s.prev_out; s.prev_out = s.cur_out; s.cur_out = t;
        t = s.prev_in; s.prev_in = s.cur_in; s.cur_in = t;
        for (int64_t v = 0; v < g->n; v++) s.cur_out[v] = s.cur_in[v] = NAN;
        if (it >= max_iterations) break;                                 /* terminate :93-95 */
    }
    if (iterations_out) *iterations_out = it;
    free(s.edge_count); free(s.prev_out); free(s.prev_in); free(s.cur_out); free(s.cur_in);
    return FR_OK;
}

/* ---- OLAPTest.DegreeCounter (tmain/olap/OLAPTest.java:334-416) ---- */
typedef struct {
    int iteration, length;
    int32_t* deg; int32_t* prev; int32_t* cur; uint8_t* prev_ok; uint8_t* cur_ok;
} dc_t;
/* DEG_MSG = inE: a row walks its OUT entries; messages summed as Java ints (wrap).  For a
 * representative row of a vertex cut this is the ADDITION combiner (:337). */
static uint32_t dc_row(const dc_t* s, const fr_graph* g, int64_t kb, int64_t ke, int* any) {
    uint32_t sum = 0;
    for (int64_t k = kb; k < ke; k++) {
        if (g->edir[k] != 0) continue;
        int64_t o = entry_vertex(g, k);
        if (o < 0 || !s->prev_ok[o]) continue;
        sum += (uint32_t)s->prev[o];
        *any = 1;
    }
    return sum;
}
static void dc_exec(void* p, const fr_graph* g, int64_t lo, int64_t hi) {
    dc_t* s = (dc_t*)p;
    for (int64_t v = lo; v < hi; v++) {
        if (s->iteration == 0) { s->cur[v] = 1; s->cur_ok[v] = 1; continue; }   /* :358-359 */
        uint32_t sum = 0;                                                /* Java int, wraps (:361) */
        int any = 0;
        /* a vertex cut sums each row's combined message into its aggregate (same Integer
         * sum, FulgoraVertexMemory.aggregateMessage :138-140) and executes once on it */
        for (int64_t i = 0; i < nrows_of(g, v); i++) {
            int64_t kb, ke; row_range(g, v, i, &kb, &ke);
            sum += dc_row(s, g, kb, ke, &any);
        }
        s->deg[v] = (int32_t)sum;                                        /* :362 */
        if (s->iteration < s->length) { s->cur[v] = (int32_t)sum; s->cur_ok[v] = 1; }   /* :363 */
    }
}
int fr_degree_counter(const fr_graph* g, int length, int threads, int32_t* out, int* iterations_out) {
    if (length <= 0) return FR_E_INVALID;                                /* :347 checkArgument */
    dc_t s; memset(&s, 0, sizeof s);
    s.length = length; s.deg = out;
    s.prev = (int32_t*)calloc(g->n + 1, 4); s.cur = (int32_t*)calloc(g->n + 1, 4);
    s.prev_ok = (uint8_t*)calloc(g->n + 1, 1); s.cur_ok = (uint8_t*)calloc(g->n + 1, 1);
    for (int64_t v = 0; v < g->n; v++) out[v] = 0;
    int it;
    for (it = 0;; it++) {
        s.iteration = it;
        superstep(g, threads, &s, dc_exec);
        int32_t* t = s.prev; s.prev = s.cur; s.cur = t;
        uint8_t* u = s.prev_ok; s.prev_ok = s.cur_ok; s.cur_ok = u;
        memset(s.cur_ok, 0, g->n + 1);
        if (it >= length) break;                                         /* terminate :368-370 */
    }
    if (iterations_out) *iterations_out = it;
    free(s.prev); free(s.cur); free(s.prev_ok); free(s.cur_ok);
    return FR_OK;
}

/* ---- Generic message passing (the primitives behind any VertexProgram) ----
 * Local scope: VertexMemoryHandler.receiveMessages (VertexMemoryHandler.java:77-93) streams
 * edgeFct(msg, e) over the reversed incident traversal (FulgoraUtil.java:57) for every
 * neighbour holding a message (null filtered); the program reduces the stream with its
 * combiner.  Here: the fold in entry order over all of the vertex's rows (a vertex cut's
 * representative rows are combined with the same combiner, FulgoraVertexMemory.java:121-147).
 * Global scope: VertexState.addMessage (VertexState.java:63-78) folds each message into the
 * target's state as it arrives: combine(message, current), in send order. */
static inline int64_t g_combine_i(int comb, int64_t acc, int64_t m) {
    if (comb == 1) return m < acc ? m : acc;
    if (comb == 2) return m > acc ? m : acc;
    return (int64_t)((uint64_t)m + (uint64_t)acc);
}
static inline double g_combine_d(int comb, double acc, double m) {
    if (comb == 1) return m < acc ? m : acc;
    if (comb == 2) return m > acc ? m : acc;
    return m + acc;
}
/* The edge functions "m op w" (w = e.value(weight)) in Java arithmetic: long + - * wrap,
 * long / truncates (MIN_VALUE / -1 = MIN_VALUE, / 0 throws ArithmeticException), double ops
 * are IEEE; a Float weight is widened to double (and refused with long messages).
 * Returns 0, or FR_E_PROGRAM for a division by zero. */
static int edge_fn_i(int fn, int64_t m, int64_t w, int64_t* out) {
    uint64_t u = (uint64_t)m;
    switch (fn) {
    case 0: *out = m; return 0;
    case 1: *out = (int64_t)(u + 1u); return 0;
    case 2: *out = (int64_t)(u + (uint64_t)w); return 0;
    case 3: *out = (int64_t)(u * (uint64_t)w); return 0;
    case 4: *out = (int64_t)(u - (uint64_t)w); return 0;
    case 5: *out = w < m ? w : m; return 0;
    case 6: *out = w > m ? w : m; return 0;
    default:
        if (w == 0) return FR_E_PROGRAM;
        *out = w == -1 ? (int64_t)(0u - u) : m / w;
        return 0;
    }
}
static double edge_fn_d(int fn, double m, double x) {
    switch (fn) {
    case 0: return m;
    case 1: return m + 1.0;
    case 2: return m + x;
    case 3: return m * x;
    case 4: return m - x;
    case 5: return x < m ? x : m;
    case 6: return x > m ? x : m;
    default: return m / x;
    }
}
/* Edge-function programs (edge_fn 8): the BiFunction<M, Edge, M> written as a postfix program
 * over m, w = e.value(weight) and constants (the op codes of include/titan_gpu_olap.h
 * tgo_edge_op).  Evaluated here in plain Java semantics, one entry at a time: long + - * and
 * negation wrap, / and % truncate, / 0 and % 0 throw ArithmeticException, Long.MIN_VALUE / -1
 * wraps to MIN_VALUE and % -1 gives 0, Math.abs(MIN_VALUE) = MIN_VALUE; double ops are IEEE,
 * % is fmod, Math.min / Math.max / Math.abs with Java's NaN and signed-zero rules.  One program
 * per process (fr_set_edge_program), set by the test before the gathers it checks. */
static struct { int n, uses_w; int32_t ops[64]; int64_t ic[64]; double fc[64]; } g_prog;
int fr_set_edge_program(const int32_t* ops, int n, const int64_t* iconsts, const double* fconsts, int nconsts) {
    if (n < 1 || n > 64 || nconsts < 0 || nconsts > 64) return FR_E_INVALID;
    g_prog.n = n; g_prog.uses_w = 0;
    for (int i = 0; i < n; i++) { g_prog.ops[i] = ops[i]; if ((ops[i] & 0xFF) == 1) g_prog.uses_w = 1; }
    for (int i = 0; i < nconsts; i++) {
        g_prog.ic[i] = iconsts ? iconsts[i] : 0;
        g_prog.fc[i] = fconsts ? fconsts[i] : 0.0;
    }
    return FR_OK;
}
static double java_min_d(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && signbit(b)) return b;
    return a <= b ? a : b;
}
static double java_max_d(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0 && signbit(a)) return b;
    return a >= b ? a : b;
}
/* 0 or FR_E_PROGRAM (an ArithmeticException) */
static int prog_eval_i(int64_t m, int64_t w, int64_t* out) {
    int64_t st[64]; int sp = 0;
    for (int i = 0; i < g_prog.n; i++) {
        int op = g_prog.ops[i] & 0xFF, arg = g_prog.ops[i] >> 8;
        if (op == 0) { st[sp++] = m; continue; }
        if (op == 1) { st[sp++] = w; continue; }
        if (op == 2) { st[sp++] = g_prog.ic[arg]; continue; }
        if (op == 10) { st[sp - 1] = (int64_t)(0u - (uint64_t)st[sp - 1]); continue; }
        if (op == 11) { if (st[sp - 1] < 0) st[sp - 1] = (int64_t)(0u - (uint64_t)st[sp - 1]); continue; }
        int64_t b = st[--sp], a = st[sp - 1], r;
        switch (op) {
        case 3: r = (int64_t)((uint64_t)a + (uint64_t)b); break;
        case 4: r = (int64_t)((uint64_t)a - (uint64_t)b); break;
        case 5: r = (int64_t)((uint64_t)a * (uint64_t)b); break;
        case 6: if (b == 0) return FR_E_PROGRAM; r = b == -1 ? (int64_t)(0u - (uint64_t)a) : a / b; break;
        case 7: if (b == 0) return FR_E_PROGRAM; r = b == -1 ? 0 : a % b; break;
        case 8: r = a <= b ? a : b; break;
        default: r = a >= b ? a : b; break;
        }
        st[sp - 1] = r;
    }
    *out = st[0];
    return 0;
}
static double prog_eval_d(double m, double w) {
    double st[64]; int sp = 0;
    for (int i = 0; i < g_prog.n; i++) {
        int op = g_prog.ops[i] & 0xFF, arg = g_prog.ops[i] >> 8;
        if (op == 0) { st[sp++] = m; continue; }
        if (op == 1) { st[sp++] = w; continue; }
        if (op == 2) { st[sp++] = g_prog.fc[arg]; continue; }
        if (op == 10) { st[sp - 1] = -st[sp - 1]; continue; }
        if (op == 11) { st[sp - 1] = st[sp - 1] <= 0.0 ? 0.0 - st[sp - 1] : st[sp - 1]; continue; }
        double b = st[--sp], a = st[sp - 1], r;
        switch (op) {
        case 3: r = a + b; break;
        case 4: r = a - b; break;
        case 5: r = a * b; break;
        case 6: r = a / b; break;
        case 7: r = fmod(a, b); break;
        case 8: r = java_min_d(a, b); break;
        default: r = java_max_d(a, b); break;
        }
        st[sp - 1] = r;
    }
    return st[0];
}

/* e.value(key) widened to double: a Float's / Double's IEEE bits, an integral value as is */
static double weight_as_double(const fr_graph* g, int64_t w) {
    if (g->wdt == FR_DT_FLOAT) { int32_t b = (int32_t)w; float f; memcpy(&f, &b, 4); return (double)f; }
    if (g->wdt == FR_DT_DOUBLE) { double d; memcpy(&d, &w, 8); return d; }
    return (double)w;
}
/* One message edgeFct(msg[o], e) of entry k (VertexMemoryHandler.java:83-92); 1 = present,
 * 0 = filtered (no message), <0 = the program fails. */
static int entry_message(const fr_graph* g, int64_t k, int64_t o, int value_type, int edge_fn, const void* msg,
                         int64_t* mi_out, double* md_out) {
    int64_t w = 0;
    const int needs_w = edge_fn == 8 ? g_prog.uses_w : edge_fn >= 2;
    if (needs_w) {
        if (!g->has_w[k]) return FR_E_PROGRAM;                                 /* e.value(key) throws */
        w = g->w[k];
    }
    if (value_type == 0) {
        if (needs_w && (g->wdt == FR_DT_FLOAT || g->wdt == FR_DT_DOUBLE)) return FR_E_INVALID;
        if (edge_fn == 8) return prog_eval_i(((const int64_t*)msg)[o], w, mi_out) ? FR_E_PROGRAM : 1;
        return edge_fn_i(edge_fn, ((const int64_t*)msg)[o], w, mi_out) ? FR_E_PROGRAM : 1;
    }
    if (edge_fn == 8) {
        *md_out = prog_eval_d(((const double*)msg)[o], needs_w ? weight_as_double(g, w) : 0.0);
        return 1;
    }
    *md_out = edge_fn_d(edge_fn, ((const double*)msg)[o], edge_fn >= 2 ? weight_as_double(g, w) : 0.0);
    return 1;
}
int fr_gather(const fr_graph* g, int scope, int value_type, int combiner, int edge_fn, const void* msg,
              const uint8_t* has, void* out, uint8_t* out_has) {
    int64_t* oi = (int64_t*)out; double* od = (double*)out;
    for (int64_t v = 0; v < g->n; v++) {
        int any = 0; int64_t ai = 0; double ad = 0.0;
        for (int64_t i = 0; i < nrows_of(g, v); i++) {
            int64_t kb, ke; row_range(g, v, i, &kb, &ke);
            for (int64_t k = kb; k < ke; k++) {
                if (!take(scope, g->edir[k])) continue;
                int64_t o = entry_vertex(g, k);
                if (o < 0 || !has[o]) continue;                                /* filter(m != null) */
                int64_t mi = 0; double md = 0.0;
                int rc = entry_message(g, k, o, value_type, edge_fn, msg, &mi, &md);
                if (rc < 0) return rc;
                if (value_type == 0) ai = any ? g_combine_i(combiner, ai, mi) : mi;
                else ad = any ? g_combine_d(combiner, ad, md) : md;
                any = 1;
            }
        }
        if (value_type == 0) oi[v] = ai; else od[v] = ad;
        out_has[v] = (uint8_t)any;
    }
    return FR_OK;
}
/* Local receive WITHOUT a combiner: the stream itself, per vertex in the order the
 * reference's receiveMessages yields it — its row's entries in column order (VertexMemoryHandler
 * .java:83-92).  off: n+1; vals: NULL for a sizing call.  A vertex cut that receives two or
 * more messages meets FulgoraUtil's ThrowingCombiner (:80-91): FR_E_PROGRAM. */
int fr_gather_lists(const fr_graph* g, int scope, int value_type, int edge_fn, const void* msg, const uint8_t* has,
                    int64_t* off, void* vals) {
    int64_t* vi = (int64_t*)vals; double* vd = (double*)vals;
    int64_t p = 0;
    off[0] = 0;
    for (int64_t v = 0; v < g->n; v++) {
        int64_t c = 0;
        for (int64_t i = 0; i < nrows_of(g, v); i++) {
            int64_t kb, ke; row_range(g, v, i, &kb, &ke);
            for (int64_t k = kb; k < ke; k++) {
                if (!take(scope, g->edir[k])) continue;
                int64_t o = entry_vertex(g, k);
                if (o < 0 || !has[o]) continue;
                int64_t mi = 0; double md = 0.0;
                int rc = entry_message(g, k, o, value_type, edge_fn, msg, &mi, &md);
                if (rc < 0) return rc;
                if (vals) { if (value_type == 0) vi[p] = mi; else vd[p] = md; }
                p++; c++;
            }
        }
        if (g->pv && g->pv[v] && c >= 2) return FR_E_PROGRAM;
        off[v + 1] = p;
    }
    return FR_OK;
}
int fr_combine_global(int64_t n, int value_type, int combiner, int64_t nmsgs, const int64_t* targets,
                      const void* values, void* out, uint8_t* out_has) {
    const int64_t* vi = (const int64_t*)values; const double* vd = (const double*)values;
    int64_t* oi = (int64_t*)out; double* od = (double*)out;
    for (int64_t v = 0; v < n; v++) { out_has[v] = 0; if (value_type == 0) oi[v] = 0; else od[v] = 0.0; }
    for (int64_t i = 0; i < nmsgs; i++) {
        int64_t t = targets[i];
        if (t < 0 || t >= n) continue;                                          /* no executing vertex */
        if (value_type == 0) oi[t] = out_has[t] ? g_combine_i(combiner, oi[t], vi[i]) : vi[i];
        else od[t] = out_has[t] ? g_combine_d(combiner, od[t], vd[i]) : vd[i];
        out_has[t] = 1;
    }
    return FR_OK;
}
