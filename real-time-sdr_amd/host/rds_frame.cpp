// rds_frame.cpp -- RDS frame synchronisation, block check and group parser (host side).
//
// Serial per-channel bit parsing (~36 decoded bits per 30.6 ms block) that turns the recovered
// bitstream into the receiver's visible output; it runs on the host exactly as in the reference
// (SURVEY 8(f) f1): start_frame_sync (src/rds_utilities.cpp:384-400) slides a 26-bit window over
// the bits of 15 decoding blocks, check_block (:352-381) computes the block syndrome against the
// IEC 62106 parity-check matrix and recognises offsets A, B, C, C', D, uint_copy (:313-337)
// places the 16 data bits of A/B/C/D into a 64-bit group register, isSequenceABCD (:339-350)
// tracks the last four offsets and parse (:172-199) prints PI, PTY and the Program Service name
// of type-0 groups to stderr. error_detection (:202-311, dead code in the reference) is the
// alternative bit-serial synchroniser (f4).
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

// ---------------------------------------------------------------------------------------------
// error_detection (src/rds_utilities.cpp:202-311): the reference's alternative,
// bit-serial synchroniser. It is never called by the reference program (rds.cpp runs
// start_frame_sync); it is served here so that the drop-in library covers rds_utilities.h:16
// whole, with the reference's observable behaviour, quirks included:
//   * unsynchronised, every bit prints the syndrome of the last 26 bits and the 64-bit history;
//     two offset syndromes a whole number of blocks apart (in the offset order A B C D, C' in C's
//     place) lock the block counter to the block after the second;
//   * synchronised, every 26th bit checks one block (B / C' alternatives for block 2), counts bad
//     blocks and, over each 50 blocks, drops sync when more than 40 were bad;
//   * the group register passed to parse() holds only the current block's 16 data bits (it is
//     cleared for every block), and parse() runs on the block that brings the good-block counter
//     (+2 for a good block A, +1 for any other good block, never reset) to exactly 5.
// The stderr text keeps the stream state the reference leaves (parse() switches std::cerr to hex).
namespace {

// x(z) z^10 mod g(z), g = z^10 + z^8 + z^7 + z^5 + z^4 + z^3 + 1 (0x5B9), over the low `nbits`
// bits of x taken most significant first
uint64_t crc10_syndrome(uint64_t x, int nbits) {
    constexpr uint32_t kGen = 0x5B9;
    uint32_t rem = 0;
    for (int k = nbits + 9; k >= 0; k--) {
        const uint32_t in = (k >= 10) ? static_cast<uint32_t>((x >> (k - 10)) & 1u) : 0u;
        rem = (rem << 1) | in;
        if (rem & 0x400u) rem ^= kGen;
    }
    return rem & 0x3FFu;
}

// offset words A, B, C, D, C' as received syndromes (unsynchronised search) and as checkword XOR
// masks (synchronised check), and each offset's position in the block cycle
constexpr uint64_t kSearchSyndrome[5] = {383, 14, 303, 663, 748};
constexpr uint64_t kOffsetWord[5] = {252, 408, 360, 436, 848};
constexpr int kCyclePos[5] = {0, 1, 2, 3, 2};

}  // namespace

void error_detection(uint64_t& reg, uint64_t& chars, uint64_t& output, bool& first_time, int& sync, int& prevsync,
                     int& lastseen_offset, int& rds_bit_cont, int& lastseen_offset_cont, int& block_distance,
                     int& block_number, int& block_bit_cont, int& blocks_cont, int& wrong_blocks_cont,
                     int& group_assembly_started, int& group_good_blocks_cont, const std::vector<int>& decoded_bits) {
    for (const int bit : decoded_bits) {
        reg = (reg << 1) | static_cast<uint64_t>(static_cast<int64_t>(bit));
        if (!sync) {
            const uint64_t syn = crc10_syndrome(reg, 26);
            std::cerr << "Reg Syndrome: " << syn << "    Reg: " << reg << std::endl;
            int hit = -1;
            for (int o = 0; o < 5 && hit < 0; o++)
                if (syn == kSearchSyndrome[o]) hit = o;
            if (hit >= 0) {
                if (!prevsync) {
                    lastseen_offset = hit;
                    lastseen_offset_cont = rds_bit_cont;
                    prevsync = 1;
                } else {
                    const int from = kCyclePos[lastseen_offset], to = kCyclePos[hit];
                    block_distance = (from >= to) ? to + 4 - from : to - from;
                    if (block_distance * 26 == rds_bit_cont - lastseen_offset_cont) {
                        std::cerr << "Sync State Detected" << std::endl;
                        wrong_blocks_cont = 0;
                        blocks_cont = 0;
                        block_bit_cont = 0;
                        block_number = (hit + 1) & 3;
                        group_assembly_started = 0;
                        sync = 1;
                    } else {
                        prevsync = 0;
                    }
                }
            }
        } else if (block_bit_cont < 25) {
            block_bit_cont++;
        } else {
            const uint64_t data = (reg >> 10) & 0xFFFF;
            const uint64_t expect = crc10_syndrome(data, 16);
            const uint64_t check = reg & 0x3FF;
            bool good = (check ^ kOffsetWord[block_number]) == expect;
            if (!good && block_number == 2) good = (check ^ kOffsetWord[4]) == expect;   // C'
            if (!good) wrong_blocks_cont++;
            uint64_t group = 0;   // cleared for every block (see above)
            if (block_number == 0 && good) {
                group_assembly_started = 1;
                group_good_blocks_cont++;
            }
            if (group_assembly_started) {
                if (good) {
                    group = data << (48 - 16 * block_number);
                    group_good_blocks_cont++;
                } else {
                    group_assembly_started = 0;
                }
                if (group_good_blocks_cont == 5) parse(group, chars, output, first_time);
            }
            block_bit_cont = 0;
            block_number = (block_number + 1) & 3;
            if (++blocks_cont == 50) {
                if (wrong_blocks_cont > 40) {
                    std::cerr << "Lost Sync (Got " << wrong_blocks_cont << " bad blocks on " << blocks_cont
                              << " total)" << std::endl;
                    sync = 0;
                    prevsync = 0;
                } else {
                    std::cerr << "Still Sync-ed (Got " << wrong_blocks_cont << " bad blocks on " << blocks_cont
                              << " total)" << std::endl;
                }
                blocks_cont = 0;
                wrong_blocks_cont = 0;
            }
        }
        rds_bit_cont++;
    }
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
