// errdet_driver.cpp -- test driver for error_detection (rds_utilities.h:16), the reference's
// alternative bit-serial RDS synchroniser. stdin: one line per decoding block, its decoded bits as
// 0/1 characters ("-" for a block that does not decode); each decoded block is passed in one call,
// with the state carried across calls. stderr: the function's own text; stdout: the final state.
// Built against the drop-in library's rds_frame.cpp (the test) or the reference's
// rds_utilities.cpp (tests/golden/make_errdet.py, fixture generation).
#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include "rds_utilities.h"

int main() {
    uint64_t reg = 0, chars = 0, output = 0;
    bool first_time = true;
    int sync = 0, prevsync = 0, lastseen_offset = 0, rds_bit_cont = 0, lastseen_offset_cont = 0, block_distance = 0,
        block_number = 0, block_bit_cont = 0, blocks_cont = 0, wrong_blocks_cont = 0, group_assembly_started = 0,
        group_good_blocks_cont = 0;
    std::string line;
    std::vector<int> bits;
    while (std::getline(std::cin, line)) {
        if (line == "-") continue;
        bits.clear();
        for (char c : line) bits.push_back(c == '1' ? 1 : 0);
        error_detection(reg, chars, output, first_time, sync, prevsync, lastseen_offset, rds_bit_cont,
                        lastseen_offset_cont, block_distance, block_number, block_bit_cont, blocks_cont,
                        wrong_blocks_cont, group_assembly_started, group_good_blocks_cont, bits);
    }
    std::cout << reg << ' ' << chars << ' ' << output << ' ' << first_time << ' ' << sync << ' ' << prevsync << ' '
              << lastseen_offset << ' ' << rds_bit_cont << ' ' << lastseen_offset_cont << ' ' << block_distance << ' '
              << block_number << ' ' << block_bit_cont << ' ' << blocks_cont << ' ' << wrong_blocks_cont << ' '
              << group_assembly_started << ' ' << group_good_blocks_cont << std::endl;
    return 0;
}
