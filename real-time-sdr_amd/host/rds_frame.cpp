// rds_frame.cpp -- RDS frame synchronisation, block check and group parser (host side).
//
// Serial per-channel bit parsing (~36 decoded bits per 30.6 ms block) that turns the recovered
// bitstream into the receiver's visible output; it runs on the host exactly as in the reference
// (SURVEY 8(f) f1): start_frame_sync (src/rds_utilities.cpp:384-400) slides a 26-bit window over
// the bits of 15 decoding blocks, check_block (:352-381) computes the block syndrome against the
// IEC 62106 parity-check matrix and recognises offsets A, B, C, C', D, uint_copy (:313-337)
// places the 16 data bits of A/B/C/D into a 64-bit group register, isSequenceABCD (:339-350)
// tracks the last four offsets and parse (:172-199) prints PI, PTY and the Program Service name
// of type-0 groups to stderr.
#include <cstdint>
#include <cstdio>
#include <deque>
#include <iostream>
#include <string>
#include <vector>

#include "rds_utilities.h"

namespace {

// Rows of the RDS parity-check matrix H (26 x 10, IEC 62106 Annex B), bit 9 = column 0. The rows
// follow the code's shift register: the first ten are the identity, each next row is the previous
// shifted right with the feedback 1011011100 whenever a one falls out.
struct ParityMatrix {
    uint32_t row[26];
    ParityMatrix() {
        uint32_t r = 0x200;
        for (int i = 0; i < 26; i++) {
            row[i] = r;
            r = (r >> 1) ^ ((r & 1u) ? 0x2DCu : 0u);
        }
    }
};
const ParityMatrix kH;

// syndromes of blocks carrying offset words A, B, C, C', D (IEC 62106)
constexpr uint32_t kSyndrome[5] = {0x3D8, 0x3D4, 0x25C, 0x3CC, 0x258};
const char* const kOffsetName[5] = {"A", "B", "C", "Cp", "D"};

// RBDS programme type names (index = 5-bit PTY code)
const char* const kPty[32] = {"Undefined", "News", "Information", "Sports", "Talk", "Rock", "Classic Rock",
                              "Adult Hits", "Soft Rock", "Top 40", "Country", "Oldies", "Soft", "Nostalgia",
                              "Jazz", "Classical", "Rhythm & Blues", "Soft Rhythm & Blues", "Language",
                              "Religious Music", "Religious Talk", "Personality", "Public", "College",
                              "Spanish Talk", "Spanish Music", "Hip Hop", "Unassigned", "Unassigned", "Weather",
                              "Emergency Test", "Emergency"};

uint32_t syndrome(std::vector<int>::const_iterator b) {
    uint32_t s = 0;
    for (int i = 0; i < 26; i++)
        if (b[i]) s ^= kH.row[i];
    return s;
}

// data bits [b, b+16) into 16-bit slot `block` (A = 0 ... D = 3, A most significant)
void place_block(uint64_t& reg, std::vector<int>::const_iterator b, int block) {
    const int shift = 48 - 16 * block;
    reg &= ~(static_cast<uint64_t>(0xFFFF) << shift);
    for (int i = 0; i < 16; i++) reg |= static_cast<uint64_t>(b[i] != 0) << (15 - i + shift);
}

bool abcd_window(const std::string& current, std::deque<std::string>& window) {
    window.push_back(current);
    if (window.size() > 4) window.pop_front();
    return window.size() == 4 && window[0] == "A" && window[1] == "B" && window[2] == "C" && window[3] == "D";
}

}  // namespace

void parse(const uint64_t& bytes, uint64_t& chars, uint64_t& output, bool& first_time) {
    const unsigned group_type = (bytes >> 44) & 0xF;
    const unsigned placement = (bytes >> 32) & 0x3;
    const uint16_t pi = (bytes >> 48) & 0xFFFF;
    const unsigned pty = (bytes >> 37) & 0x1F;
    std::cerr << "PI: " << std::hex << pi << std::endl;
    std::cerr << "PTY: " << kPty[pty] << std::endl;
    first_time = false;
    if (group_type == 0) {
        const int shift = 16 * (3 - static_cast<int>(placement));
        chars = (chars & ~(static_cast<uint64_t>(0xFFFF) << shift)) | ((bytes & 0xFFFF) << shift);
        if (placement == 3 && chars != output) {
            output = chars;
            char name[9];
            for (int i = 0; i < 8; i++) name[i] = static_cast<char>((chars >> (56 - 8 * i)) & 0xFF);
            name[8] = '\0';
            std::cerr << "Program Service: " << name << std::endl;
        }
    }
}

void check_block(std::string& offset_type, std::vector<int>::iterator bitstream_start,
                 std::vector<int>::iterator bitstream_end, uint64_t& reg, uint64_t& chars, uint64_t& output,
                 bool& first_time, std::deque<std::string>& window) {
    (void)bitstream_end;
    const uint32_t s = syndrome(bitstream_start);
    for (int o = 0; o < 5; o++) {
        if (s != kSyndrome[o]) continue;
        offset_type = kOffsetName[o];
        if (o != 3) place_block(reg, bitstream_start, o < 3 ? o : 3);
        if (abcd_window(offset_type, window)) parse(reg, chars, output, first_time);
        return;
    }
    offset_type = "None";
}

void start_frame_sync(unsigned int& idx, std::vector<int>& stream, std::vector<int>& sync_state_bits, uint64_t& reg,
                      uint64_t& chars, uint64_t& output, bool& first_time, std::deque<std::string>& window) {
    stream.insert(stream.begin(), sync_state_bits.begin(), sync_state_bits.end());
    // the reference scans start positions idx < size - 26 (unsigned)
    const unsigned int end_range = static_cast<unsigned int>(stream.size()) - 26u;
    std::string type;
    while (stream.size() >= 26 && idx < end_range) {
        check_block(type, stream.begin() + idx, stream.begin() + idx + 26, reg, chars, output, first_time, window);
        idx += (type != "None") ? 26 : 1;
    }
    sync_state_bits.assign(stream.begin() + idx, stream.end());
}
